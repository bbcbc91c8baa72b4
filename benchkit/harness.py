"""The one timing harness every benchmark leg runs under (bench.py's contract).

W untimed warmup steps, then exactly K timed steps bracketed by a barrier and
torch.cuda.synchronize() on both sides; the elapsed time is the max over ranks and the bytes
the sum over ranks, so ``value`` is the whole job's throughput.

Steps in flight (S > 1 contexts, each with its own stream and input) need one more rule
(VERDICT r4): a timed region of K < 2S steps starting from an empty pipeline measures a burst
(every stream starts at t0 and they end together), not a steady state.  So plan_steps raises K
to at least 2S and W to at least S, and steady_state() reports the rate over the completions
after the first S, when the pipeline was full, beside the whole-region value.
"""
import json
import time

from .common import GIB, SYNTH_DATA, med


def plan_steps(steps: int, warmup: int, inflight: int):
    """(steps, warmup, note) to run with `inflight` steps in flight: at least 2 S timed steps
    and S warmup steps when S > 1 (note says what was raised, None if nothing)."""
    S = max(1, int(inflight))
    if S == 1:
        return steps, warmup, None
    k, w = max(steps, 2 * S), max(warmup, S)
    if (k, w) == (steps, warmup):
        return k, w, None
    return k, w, ("%d steps in flight: timed steps raised %d -> %d and warmup %d -> %d so the "
                  "timed region holds two full pipelines (harness.plan_steps)"
                  % (S, steps, k, warmup, w))


def steady_state(t0: float, done_at, inflight: int, bytes_per_step: float):
    """Rate over the timed completions after the first S (the pipeline full), GiB/s; None when
    fewer than S + 1 steps completed in the timed region."""
    S, K = max(1, int(inflight)), len(done_at)
    if K <= S:
        return None
    window = done_at[-1] - done_at[S - 1]
    if window <= 0:
        return None
    return {"value": round(bytes_per_step * (K - S) / window / GIB, 3), "unit": "GiB/s",
            "steps": K - S, "ms_per_step": round(window * 1e3 / (K - S), 3),
            "note": "completions %d..%d of the timed region (the first %d fill the pipeline), "
                    "this rank" % (S + 1, K, S)}


class Harness:
    """Timing, reduction over ranks and the JSON line for one leg.  ctx: bench.py's context
    dict (torch, dist, world, rank, cdev)."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.torch, self.dist = ctx["torch"], ctx["dist"]
        self.world, self.rank, self.cdev = ctx["world"], ctx["rank"], ctx["cdev"]

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def timed(self, run, steps: int) -> float:
        """run(steps) between barrier + synchronize on both sides; seconds, max over ranks."""
        self.barrier()
        self.torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.t0 = t0
        run(steps)
        self.torch.cuda.synchronize()
        self.barrier()
        return self.max_over_ranks(time.perf_counter() - t0)

    def max_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def line(self, metric, bytes_all_ranks, steps, warmup, elapsed, scaling, config,
             data=SYNTH_DATA, dtype="u8", **extra):
        """The contract's JSON object: value = the bytes all ranks processed per step x steps /
        elapsed (GiB/s)."""
        K = max(steps, 1)
        out = {"metric": metric,
               "value": round(float(bytes_all_ranks) * steps / elapsed / GIB, 3) if elapsed else 0.0,
               "unit": "GiB/s", "n_gpus": self.world, "steps": steps, "warmup": warmup,
               "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
               "scaling": scaling, "vs_baseline": None, "dtype": dtype, "data": data,
               "config": config}
        out.update(extra)
        return out

    def emit(self, out):
        if self.rank == 0:
            print(json.dumps(out), flush=True)

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


__all__ = ["Harness", "plan_steps", "steady_state", "med"]
