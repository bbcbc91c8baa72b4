# Static VALU count of the hash kernel's two unrolled iterations (first..last ds_read_b64).
# usage: bash tools/valu_count.sh [extra hipcc flags]
f=/tmp/vc_$$.s
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o $f "$@" $(dirname $0)/../pfs_amd/csrc/cdc_kernels.hip 2>/dev/null
awk '/^_ZN6pfscdc14blake2b_kernel/,/s_endpgm/' $f > $f.k
a=$(grep -n "ds_read_b64" $f.k | head -1 | cut -d: -f1); b=$(grep -n "ds_read_b64" $f.k | tail -1 | cut -d: -f1)
sed -n "${a},${b}p" $f.k | grep -E "^\s+v_" | awk '{print $1}' | sort | uniq -c | sort -rn | head -12
echo "VALU total: $(sed -n "${a},${b}p" $f.k | grep -cE '^\s+v_')  s_nop: $(sed -n "${a},${b}p" $f.k | grep -c s_nop)"
rm -f $f $f.k
