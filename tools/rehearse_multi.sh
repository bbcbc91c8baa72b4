# N>1 bench rehearsal on a one-GPU box: every rank on device 0, gloo collectives
# (PFS_BENCH_REHEARSE=1).  Checks the sharding, index gather, max-over-ranks timing and the
# JSON line; the driver's scaling runs use one GPU per rank over RCCL.
mkdir -p gpurun_out/rehearse
export PFS_BENCH_REHEARSE=1
run() { # name nproc args...
  local name=$1 np=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $((29500 + np)) bench.py --gpus $np "$@" \
    > gpurun_out/rehearse/$name.json 2> gpurun_out/rehearse/$name.err
}
run c2_n2 2 --steps 2 --warmup 1 --group 4 --no-cpu-baseline --no-e2e && \
run c2_n4 4 --steps 2 --warmup 1 --group 2 --no-cpu-baseline --no-e2e && \
run c4_n2 2 --config c4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e && \
run c5_n2 2 --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e
rc=$?
for f in gpurun_out/rehearse/*.json; do echo "== $f"; cat $f; done
exit $rc
