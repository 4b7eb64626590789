"""bench.py -- batched SRBD-MPC QP solves/s on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic robots per GPU:
qp_former (HIP) -> cold-started sparse PDIPM (HIP, 10 Mehrotra iterations), i.e. the reference GPU
caller's QP step (biped_pympc/convex_mpc/mpc_controller_cusadi.py:99-169) at BASELINE config 2
(batch 4096, horizon N = 10, 10 PDIPM iterations) per GPU; for N > 1 ranks each GPU solves its own
4096-env shard (weak scaling) and the first-stage inputs u0 (12 doubles/env, the only thing the
wrapper consumes, mpc_controller_cusadi.py:186) are gathered over RCCL.

Usage: python bench.py [--gpus N --steps K --warmup W]   (multi-GPU via torch.distributed.run)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from biped_pympc_amd import solver  # noqa: E402
from biped_pympc_amd.layout import Dims  # noqa: E402
from biped_pympc_amd.sharding import ShardedMPC  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

# Structural work per solve, frozen from scripts/algorithmic_work.py (SURVEY.md 8d convention:
# the reference's sparse LDL^T of its 70N KKT per iteration; bytes = algorithmic HBM traffic).
# bytes_fused = former inputs in + x, s, z, y, residuals, mu out (BASELINE.md "fused" bytes/solve).
WORK = {
    10: {"flops_per_iter": 75840, "bytes_pdipm_cold": 23688, "bytes_step": 45352,
         "bytes_former": 3616 + 18048, "bytes_fused": 3616 + 5640},
    20: {"flops_per_iter": 165074, "bytes_pdipm_cold": 47528, "bytes_step": 90472,
         "bytes_former": 6656 + 36288, "bytes_fused": 6656 + 11240},
}
PEAK_FP64_TFLOPS = 78.6  # MI355X FP64 vector = FP64 matrix peak (AMD spec; no sparsity)
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
NODE_GPUS = int(os.environ.get("SRBD_NODE_GPUS", "8"))  # GPUs sharing one host (an 8-GPU MI355X node)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch-per-gpu", type=int, default=4096)
    p.add_argument("--horizon", type=int, default=10)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--random-gait", action="store_true")
    p.add_argument("--kernel-reps", type=int, default=10)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-full-host", action="store_true",
                   help="also time the CPU baseline on every CPU the process may run on (off by default: "
                        "the GPU box gives one GPU's job a 16-CPU share of the host)")
    p.add_argument("--no-controller", action="store_true", help="skip the controller-step timing (PMC passes)")
    return p.parse_args()


def event_time_ms(fn, reps: int, warm: int = 2) -> float:
    """Average duration of fn() on torch's current stream (where the kernels are launched), after
    `warm` untimed calls (first-launch attribute setup, clock ramp)."""
    s = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def reg_horizon(N: int) -> bool:
    """Horizons with a register-resident kernel (csrc/pdipm_srbd_reg.hpp reg_horizon)."""
    return 2 <= N <= 32


def solver_kernel_name(N: int) -> str:
    """The kernel that runs the bench step at horizon N (srbd_mpc_solve_fused, one launch): the
    register-resident fused former + solver kernel, or the LDS-resident step kernel at the other
    horizons."""
    return f"mpc_step_reg_kernel<{N}>" if reg_horizon(N) else "mpc_step_lds_kernel<0>"


def load_pmc(N: int, B: int, K: int):
    """HBM bytes per solver launch from the committed rocprofv3 --pmc summary of this kernel (the
    latest round's profiles/ first)."""
    name = solver_kernel_name(N)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (d.get("horizon") == N and d.get("batch") == B and d.get("iters") == K
                and name in (d.get("kernel") or "")):
            return d.get("pdipm_hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def load_sq(N: int, B: int, K: int):
    """VALU / LDS busy shares of the bench kernel from the committed rocprofv3 SQ-counter summary
    (scripts/gpu_sq_counters.sh + scripts/sq_summary.py --json)."""
    name = solver_kernel_name(N)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "sq_counters_*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (d.get("horizon") == N and d.get("batch") == B and d.get("iters") == K
                and name in (d.get("kernel") or "") and d.get("utilisation")):
            return dict(d["utilisation"], source=f"from {os.path.relpath(path, ROOT)} (rocprofv3 SQ counters, offline)")
    return None


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _physical_cores(cpus) -> int:
    """Distinct (package, core) pairs among the logical CPUs `cpus` (SMT siblings count once)."""
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            with open(base + "physical_package_id") as f1, open(base + "core_id") as f2:
                seen.add((f1.read().strip(), f2.read().strip()))
        except OSError:
            seen.add(("?", str(c)))
    return len(seen)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # rehearsal hooks for the N > 1 path on a one-GPU box (never set by the driver): all ranks on
    # device 0, and gloo instead of RCCL (RCCL rejects two ranks on one device)
    one_device = os.environ.get("SRBD_BENCH_ONE_DEVICE") == "1"
    backend = os.environ.get("SRBD_BENCH_BACKEND", "nccl")
    if one_device:
        local = 0
    if world > 1:
        import torch.distributed as dist_mod
        dist = dist_mod
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    N, K, B = a.horizon, a.iters, a.batch_per_gpu
    d = Dims(N)

    # each rank's shard of the global synthetic batch (world x B robots) is generated locally
    wl = make_workload(B, N, seed=1000 + rank, random_gait=a.random_gait)
    inputs = [torch.from_numpy(x).to(dev) for x in wl.inputs]
    sh = ShardedMPC(N, K, world * B, device=dev, y0=1.0)

    # per-kernel timing (HIP events on the launch stream) BEFORE the timed steps, on buffers of their
    # own: the driver's short runs (--warmup 5) otherwise time the first steps while the GPU's clocks
    # are still ramping up from idle (round 2: 0.687 ms per step at 20 steps vs 0.664 ms at 100)
    bufs = solver.MPCSolveBuffers.allocate(N, B, dev)
    qp = bufs.qp_views()
    sol_qp = [qp[0], qp[4], qp[2], qp[1], qp[5], qp[3]]  # H, G, A, f, h(=d), b
    pd_out = solver._alloc_solver_outputs(B, N, dev)
    ms_former = event_time_ms(lambda: solver.qp_former(inputs, N, outputs=qp), a.kernel_reps)
    ms_pdipm = event_time_ms(lambda: solver.pdipm(sol_qp, None, N, K, 1.0, outputs=pd_out),
                             a.kernel_reps)
    # the step's own kernel: fused former + solver (one launch at every horizon), on the same inputs
    ms_fused = event_time_ms(lambda: solver.mpc_solve(inputs, N, K, 1.0, buffers=bufs), a.kernel_reps)
    del pd_out

    pending = []

    def step():
        if world == 1:
            return sh.step(inputs)  # fused former + PDIPM
        # shard solve; the u0 gather (RCCL) runs on its own stream, overlapping the next step
        pending.append(sh.step_async(inputs))

    def drain():  # every gather of the timed steps completes inside the timed region
        for h in pending:
            h.wait()
        pending.clear()

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = 1e3 * elapsed / a.steps
    value = world * B * a.steps / elapsed

    # the step's kernel timed again at steady clocks (the legs above also serve as the clock warm-up);
    # roofline.achieved uses this figure
    ms_fused = event_time_ms(lambda: solver.mpc_solve(inputs, N, K, 1.0, buffers=bufs), a.kernel_reps)
    fused = True  # srbd_mpc_solve_fused is one launch at every horizon
    ms_main = ms_fused
    # the whole controller step: input prep + former + PDIPM + wrench in ONE launch
    # (srbd_mpc_step) vs the same three stages as three launches, on B synthetic robots
    ctrl = None
    if not a.no_controller:
        from biped_pympc_amd.utils.synthetic import make_controller
        c = make_controller(B, N, seed=77 + rank, device=dev, n_iter=K)

        def ab(cc):  # one launch vs three launches, interleaved so clock drift hits both alike
            ones, threes = [], []
            for _ in range(3):
                ones.append(event_time_ms(cc.run, a.kernel_reps))
                threes.append(event_time_ms(cc.run_three_kernel, a.kernel_reps))
            return sum(ones) / 3, sum(threes) / 3
        ms_one, ms_three = ab(c)
        ctrl = {"one_launch_ms": round(ms_one, 4), "three_kernel_ms": round(ms_three, 4),
                "robots_per_s": round(B / (ms_one * 1e-3), 1),
                "bytes_out_per_env": 48, "note": "prep + former + PDIPM + wrench; wrench-only output"}
        c256 = make_controller(256, N, seed=78 + rank, device=dev, n_iter=K)
        m1, m3 = ab(c256)
        ctrl["b256"] = {"one_launch_ms": round(m1, 4), "three_kernel_ms": round(m3, 4)}
        del c, c256
    ms_gather = None
    if dist is not None:
        u0 = bufs.outputs[0][:, 12 * N:12 * N + 12]
        ms_gather = event_time_ms(lambda: sh.gather_u0(u0), a.kernel_reps)

    w = WORK.get(N)
    roofline = None
    if w is not None:
        flops = w["flops_per_iter"] * K * B
        achieved = flops / (ms_main * 1e-3) / 1e12
        hbm_bytes = (w["bytes_fused"] if fused else w["bytes_pdipm_cold"]) * B
        traffic, traffic_src = load_pmc(N, B, K)
        roofline = {
            "bound": "fp64-valu", "kernel": solver_kernel_name(N), "achieved": round(achieved, 4),
            "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP64_TFLOPS, 6),
            # traffic and utilisation are NOT measured in this run: they are read from the committed
            # rocprofv3 --pmc / SQ-counter summaries of the same kernel and configuration
            "traffic": traffic, "traffic_source": traffic_src and f"from {traffic_src} (rocprofv3 --pmc, offline)",
            "algorithmic_flops_per_launch": flops, "launch_ms": round(ms_main, 4),
            "note": ("FP64 compute roof (vector == matrix peak on MI355X); the kernel runs on the "
                     "FP64 VALU (no MFMA): bound = its issue rate and the 12x12 chains. Flops = the reference's sparse-LDL KKT work per iteration "
                     "(SURVEY 8d) x iterations x QPs per launch. Bytes = former inputs in + "
                     "solution out per QP (fused step)." if fused else
                     "FP64 compute roof; flops as SURVEY 8d; bytes = QP in + solution out."),
            "utilisation": load_sq(N, B, K),  # VALU / LDS busy shares from profiles/ (SQ counters, offline)
            "hbm": {"achieved_GBs": round(hbm_bytes / (ms_main * 1e-3) / 1e9, 2),
                    "peak_GBs": PEAK_HBM_GBS,
                    "frac": round(hbm_bytes / (ms_main * 1e-3) / 1e9 / PEAK_HBM_GBS, 6),
                    "algorithmic_bytes_per_launch": hbm_bytes},
        }

    cpu = None
    parity = None
    if rank == 0 and not a.no_cpu_baseline:
        from oracle import oracle  # cpu_baseline leg: the oracle as baseline and checker only
        host_cpus = os.cpu_count() or 1
        affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host_cpus
        # OpenMP over envs on this process's CPU share: OMP_NUM_THREADS where the harness sets it
        # (the GPU box gives one GPU's job 16 CPUs of a larger host), else every CPU it may run on
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or affinity
        sample = min(B, 512)
        sub = [x[:sample] for x in wl.inputs]
        oracle.mpc_solve(N, K, [x[:8] for x in sub], nthreads=threads)  # symbolic setup + warm
        for _ in range(3):  # SURVEY 8(d) protocol: 3 warm-up calls, then timed repeats (>= 20)
            oracle.mpc_solve(N, K, sub, y0=1.0, nthreads=threads)
        solves, t_cpu, ref, passes = 0, 0.0, None, []
        while t_cpu < a.cpu_seconds or len(passes) < 20:
            t1 = time.perf_counter()
            ref = oracle.mpc_solve(N, K, sub, y0=1.0, nthreads=threads)
            dt = time.perf_counter() - t1
            passes.append(dt)
            t_cpu += dt
            solves += sample
        q1, med, q3 = np.percentile(sample / np.array(passes), [25, 50, 75])
        aff_cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(host_cpus))
        phys_host = _physical_cores(range(host_cpus))
        phys_aff = _physical_cores(aff_cpus)
        cores_used = min(threads, phys_aff)  # OpenMP threads spread over distinct physical cores first
        full = None
        if a.cpu_full_host:  # measured on every CPU of the affinity set (opt-in, see --help)
            oracle.mpc_solve(N, K, sub, y0=1.0, nthreads=affinity)
            nf, tf = 0, 0.0
            while tf < a.cpu_seconds / 2:
                t1 = time.perf_counter()
                oracle.mpc_solve(N, K, sub, y0=1.0, nthreads=affinity)
                tf += time.perf_counter() - t1
                nf += sample
            full = {"value": round(nf / tf, 1), "threads": affinity, "physical_cores": phys_aff}
        # BASELINE config 1 (B = 1, N = 10, K = 5: the reference's CPU-runnable case) on one core,
        # and B = 256 at the bench's K on the same CPU share
        one = [x[:1] for x in wl.inputs]
        n1, t1s = 0, 0.0
        while t1s < 1.0:
            t1 = time.perf_counter()
            oracle.mpc_solve(N, 5, one, y0=1.0, nthreads=1)
            t1s += time.perf_counter() - t1
            n1 += 1
        sub256 = [x[:256] for x in wl.inputs]
        t1 = time.perf_counter()
        oracle.mpc_solve(N, K, sub256, y0=1.0, nthreads=threads)
        t256 = time.perf_counter() - t1
        cpu = {"value": round(solves / t_cpu, 1), "unit": "solves/s", "cores": threads,
               "median": round(float(med), 1), "iqr": [round(float(q1), 1), round(float(q3), 1)],
               "kind": "port", "per_core": round(solves / t_cpu / cores_used, 1),
               "per_core_basis": f"{cores_used} physical cores ({threads} OpenMP threads)",
               "host": {"logical_cpus": host_cpus, "physical_cores": phys_host, "affinity_cpus": affinity,
                        "affinity_physical_cores": phys_aff, "model": _cpu_model(),
                        # one GPU's fair share of the host's physical cores, and the whole host, at the
                        # measured per-core rate (linear scaling assumed: the envs are independent)
                        "per_gpu_share_estimate": round(solves / t_cpu / cores_used * phys_host / NODE_GPUS, 1),
                        "node_gpus": NODE_GPUS,
                        "full_host_estimate": round(solves / t_cpu / cores_used * phys_host, 1),
                        "full_host_measured": full},
               "sample": (f"C oracle (full-KKT sparse LDL^T PDIPM, OpenMP over envs, {threads} threads) on "
                          f"the first {sample} envs of the same workload, {solves // sample} passes, "
                          f"{t_cpu:.1f} s, N={N}, {K} iterations"),
               "config1_b1_k5": {"ms_per_solve": round(1e3 * t1s / n1, 4), "cores": 1},
               "b256": {"solves_per_s": round(256 / t256, 1), "cores": threads, "iters": K}}
        # GPU latency of the same two small configurations (one launch each, resident inputs)
        g1 = [t[:1].contiguous() for t in inputs]
        g256 = [t[:256].contiguous() for t in inputs]
        cpu["config1_b1_k5"]["gpu_ms"] = round(event_time_ms(lambda: solver.mpc_solve(g1, N, 5, 1.0), a.kernel_reps), 4)
        cpu["b256"]["gpu_ms"] = round(event_time_ms(lambda: solver.mpc_solve(g256, N, K, 1.0), a.kernel_reps), 4)
        x = solver.mpc_solve([t[:sample].contiguous() for t in inputs], N, K, 1.0)[0]
        torch.cuda.synchronize()
        x = x.cpu().numpy()
        ug, ur = x[:, 12 * N:12 * N + 12], ref[0][:, 12 * N:12 * N + 12]
        du = np.abs(ug - ur)
        parity = {"max_abs_du": float(du.max()),
                  "max_rel_du": float((du.max(axis=1) / np.abs(ur).max(axis=1)).max()),
                  "envs": sample, "vs": "oracle (CPU restatement; CasADi unavailable: parity unpinned)"}
    if dist is not None:
        dist.barrier()  # the other ranks wait for rank 0's CPU leg before tearing down

    if rank == 0:
        line = {
            "metric": "batched SRBD QP solves/sec (N=10, 10 PDIPM iters)" if (N, K) == (10, 10)
            else f"batched SRBD QP solves/sec (N={N}, {K} PDIPM iters)",
            "value": round(value, 1), "unit": "solves/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"SRBD MPC QP step: qp_former + {K}-iteration sparse PDIPM, "
                                   f"batch {B}/GPU, horizon N={N}"
                                   + (", randomized gait" if a.random_gait else ", standing gait"),
                       "batch_per_gpu": B, "global_batch": B * world, "horizon": N,
                       "pdipm_iters": K, "qp_dims": [d.nz, d.n_eq, d.n_ineq],
                       "parallelism": f"dp{world}" + (f" (u0 all_gather over {'RCCL' if backend == 'nccl' else backend})"
                                                      if world > 1 else "")},
            # solves/s without the u0 gather (every rank's shard solve alone), N > 1 only
            "value_without_gather": (round(world * B / (ms_main * 1e-3), 1) if dist is not None else None),
            "kernels_ms": {"mpc_step_fused": round(ms_fused, 4) if fused else None,
                           "qp_former": round(ms_former, 4), "pdipm": round(ms_pdipm, 4),
                           "u0_all_gather": None if ms_gather is None else round(ms_gather, 4)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
            "controller_step": ctrl,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
