#!/bin/bash
# round 3: which part of the scan sets its clock (timing-only builds: wrong results)
timeout -k 10 600 bash tools/ab_clock.sh 2 pfs_amd/libpfscdc.so pfs_amd/libpfscdc_x_notable.so pfs_amd/libpfscdc_x_norot.so pfs_amd/libpfscdc_x_noperm.so
