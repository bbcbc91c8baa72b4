# A/B timing of scan-kernel experiment builds (timing only; outputs of EXP builds are wrong)
mkdir -p gpurun_out; : > gpurun_out/ab.txt
for v in "" ${@}; do
  lib=pfs_amd/libpfscdc${v:+_$v}.so
  PFSCDC_LIB=$PWD/$lib timeout -k 10 120 python tools/prof_driver.py 4 8192 >> gpurun_out/ab.txt 2>&1 && echo "^ $lib" >> gpurun_out/ab.txt
done
echo rc=$?
