#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/rehearse_r4_n4.sh &&
bash tools/r4_session12.sh
