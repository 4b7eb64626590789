"""bench.py -- batched SRBD-MPC QP solves/s on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic robots per GPU:
qp_former (HIP) -> cold-started sparse PDIPM (HIP, 10 Mehrotra iterations), i.e. the reference GPU
caller's QP step (biped_pympc/convex_mpc/mpc_controller_cusadi.py:99-169) at BASELINE config 2
(batch 4096, horizon N = 10, 10 PDIPM iterations) per GPU; for N > 1 ranks each GPU solves its own
4096-env shard (weak scaling) and the first-stage inputs u0 (12 doubles/env, the only thing the
wrapper consumes, mpc_controller_cusadi.py:186) are gathered over RCCL.

Usage: python bench.py [--gpus N --steps K --warmup W]
  --gpus N > 1 without an external launcher: this process starts N ranks itself (one child process
  per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their
  environment), touches no GPU itself, and exits with the first failing rank's status. Under
  torch.distributed.run (WORLD_SIZE set) --gpus must equal WORLD_SIZE, else it exits 2.
Prints ONE JSON line on rank 0; n_gpus = the ranks that joined the process group.
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

from biped_pympc_amd import _native, solver  # noqa: E402
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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU; default: WORLD_SIZE under an external launcher, else 1); > 1 "
                        "without WORLD_SIZE set: bench.py starts them itself")
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
    p.add_argument("--no-dropin", action="store_true",
                   help="skip the reference caller's CusADi schedule leg (1 former + 4 x 5-iteration evaluate)")
    p.add_argument("--sustain-seconds", type=float, default=8.0,
                   help="after the timed steps, run the step kernel back to back for this long (0: skip)")
    p.add_argument("--no-config3", action="store_true",
                   help="skip the BASELINE config-3 leg (fused N = 20, B = 4096, K = 10 kernel + oracle sample)")
    p.add_argument("--dump-u0", default=None,
                   help="rank 0 saves the gathered u0 (global env order) of the last timed step as .npy")
    return p.parse_args(argv)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv) -> int:
    """Start a.gpus ranks of this script (one process per GPU) and wait for them.

    The parent imports nothing that touches the GPU and never execs: each rank is a child process
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as torch.distributed.run
    would set them. Rank 0's stdout (the JSON line) is this process's stdout; the other ranks'
    stdout is dropped, every rank's stderr is kept. If a rank fails, the others are terminated
    (a rank left waiting in a collective would otherwise hang) and its exit status is returned."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = {s: signal.signal(s, lambda *x, s=s: (stop(), sys.exit(128 + s))) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            for r, p in enumerate(procs):
                code = p.poll()
                if code not in (None, 0) and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank {r} exited with status {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    stop()
            time.sleep(0.1)
        for r, p in enumerate(procs):
            if p.returncode not in (0, None) and rc == 0:
                rc = p.returncode if p.returncode > 0 else 128 - p.returncode
    finally:
        stop()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def load_solve_hook(spec: str):
    """SRBD_BENCH_SOLVE_HOOK="module:factory" -- test hook (never set by the driver): the step's
    solve becomes factory(N, K)(local_inputs) -> x on the CPU and every GPU leg is skipped, so the
    launcher, the process group and the u0 gather run on a machine without a GPU (tests/)."""
    import importlib
    mod, _, attr = spec.partition(":")
    return getattr(importlib.import_module(mod), attr)


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


def _cgroup_cpu_quota():
    """CPUs this process may use per the cgroup v2 CPU controller (cpu.max "quota period"), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


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


def run_timed(sh, inputs, a, dist, world, dev):
    """W untimed warm-up steps, then EXACTLY a.steps steps bracketed by a barrier + device sync on
    both sides; returns (max over ranks of the elapsed seconds, u0 of every env after the last step).
    At world > 1 each step leaves its u0 gather running on the collective's stream (overlapping the
    next step's solve) and every gather completes inside the timed region."""
    cuda = dev.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    pending = []
    last = [None]

    def step():
        if world == 1:
            last[0] = sh.step(inputs)  # fused former + PDIPM
        else:
            pending.append(sh.step_async(inputs))

    def drain():
        for h in pending:
            last[0] = h.wait()
        pending.clear()

    for _ in range(a.warmup):
        step()
    drain()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = own = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, last[0], own


def rank_spread(dist, dev, solve_ms: float, gather_ms: float, elapsed_s: float):
    """Per-rank figures of an N > 1 run, gathered to every rank: each rank's shard solve (its own
    step kernel, timed alone), its u0 gather (timed alone) and its own clock over the timed steps, so
    a sub-linear point can be attributed to a slow rank or to the gather. None without a group."""
    if dist is None:
        return None
    world = dist.get_world_size()
    mine = torch.tensor([solve_ms, gather_ms, 1e3 * elapsed_s], dtype=torch.float64, device=dev)
    every = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    v = torch.stack(every).cpu().numpy()
    return {"joined": world,
            "solve_ms_min": round(float(v[:, 0].min()), 4), "solve_ms_max": round(float(v[:, 0].max()), 4),
            "slowest_solve_rank": int(v[:, 0].argmax()),
            "gather_ms_max": round(float(v[:, 1].max()), 4),
            "timed_ms_min": round(float(v[:, 2].min()), 3), "timed_ms_max": round(float(v[:, 2].max()), 3),
            "solve_ms_per_rank": [round(float(x), 4) for x in v[:, 0]],
            "gather_ms_per_rank": [round(float(x), 4) for x in v[:, 1]]}


def hook_main(a, hook, dist, world, rank, N, K, B, d):
    """The launcher / process-group / gather path with a CPU solve (SRBD_BENCH_SOLVE_HOOK): same
    workload seeds and timing as main(), no GPU leg; the line says which solve ran."""
    dev = torch.device("cpu")
    wl = make_workload(B, N, seed=1000 + rank, random_gait=a.random_gait)
    inputs = [torch.from_numpy(x) for x in wl.inputs]
    solve = load_solve_hook(hook)(N, K)
    sh = ShardedMPC(N, K, world * B, device=dev, y0=1.0, solve_fn=solve)
    elapsed, u0_last, own = run_timed(sh, inputs, a, dist, world, dev)
    t1 = time.perf_counter()
    x = solve(inputs)
    solve_ms = 1e3 * (time.perf_counter() - t1)
    t1 = time.perf_counter()
    sh.gather_u0(x[:, 12 * N:12 * N + 12])
    ranks = rank_spread(dist, dev, solve_ms, 1e3 * (time.perf_counter() - t1), own)
    if rank == 0:
        if a.dump_u0:
            np.save(a.dump_u0, u0_last.numpy())
        emit({
            "metric": f"batched SRBD QP solves/sec (N={N}, {K} PDIPM iters)", "value": round(world * B * a.steps / elapsed, 1),
            "unit": "solves/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"CPU solve hook {hook} (launcher test; not a GPU measurement)",
                       "batch_per_gpu": B, "global_batch": B * world, "horizon": N, "pdipm_iters": K,
                       "parallelism": f"dp{world}" + (" (u0 all_gather over gloo)" if world > 1 else "")},
            "ranks": ranks})
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _claim_stdout():
    """The JSON line is the only thing on stdout: native libraries (gloo, RCCL, HIP) print
    diagnostics to file descriptor 1, so fd 1 is pointed at stderr and the line goes to a private
    duplicate of the original stdout."""
    global OUT
    sys.stdout.flush()
    OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


OUT = sys.stdout


def emit(line: dict) -> None:
    print(json.dumps(line), file=OUT, flush=True)


def dropin_leg(inputs, N: int, B: int, reps: int) -> dict:
    """The reference caller's own schedule through the CusADi-ABI drop-in libraries
    (mpc_controller_cusadi.py:99-172: 1 former evaluate, 4 x 5-iteration solver evaluate, blocking,
    with the dense rebuilds and clones between calls), timed on the host clock because every
    evaluate blocks, beside the one-launch fused step with the same 20 iterations."""
    from biped_pympc_amd.cusadi.reference_step import ReferenceQPSchedule
    out = {}
    xs = {}
    for name, lean in (("literal", False), ("lean", True)):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        sched = ReferenceQPSchedule(N, B, lean=lean)
        xs[name] = sched.run(inputs)  # warm: library load, attribute setup
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(max(2, reps // 2)):
            sched.run(inputs)
        torch.cuda.synchronize()
        out[f"{name}_ms"] = round(1e3 * (time.perf_counter() - t0) / max(2, reps // 2), 4)
        # device memory the leg allocated at its peak (CusadiFunction buffers + the schedule's
        # temporaries), above what was allocated before it
        out[f"{name}_peak_mb"] = round((torch.cuda.max_memory_allocated() - base) / 2**20, 1)
        del sched
    bufs = solver.MPCSolveBuffers.allocate(N, B, inputs[0].device)
    out["fused_k20_ms"] = round(event_time_ms(lambda: solver.mpc_solve(inputs, N, 20, 1.0, buffers=bufs), reps), 4)
    x20 = bufs.outputs[0]
    for name, x in xs.items():
        out[f"{name}_vs_fused_max_rel"] = float(((x - x20).abs().amax(dim=1) / x20.abs().amax(dim=1)).max())
    out["note"] = ("MPCControllerCusadi.run's QP schedule (INTEGRATION.md option A): 1 former + 4 x 5-iteration "
                   "evaluate, blocking, through CusadiFunction; 'literal' keeps the reference's dense "
                   "getDenseOutput rebuilds, bmm init and clones, 'lean' feeds the sparse outputs back; "
                   "fused_k20 = the same 20 Newton iterations as one srbd_mpc_solve_fused launch; *_peak_mb = the "
                   "leg's peak device memory above the bench's own (CusadiFunction.outputs_dense is allocated "
                   "only when read, so the never-written dense outputs hold no HBM)")
    return out


C3_N, C3_B, C3_K, C3_SAMPLE = 20, 4096, 10, 64


def sustained_leg(fn, B: int, seconds: float, burst: int = 250) -> dict:
    """The step kernel back to back for `seconds` in bursts of `burst` launches, each burst timed with
    HIP events on the launch stream: the steady-state rate (clocks and power settled, no idle gaps) and
    the spread over bursts. Also gives the driver's GPU-activity sampler a window of real load."""
    per = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        per.append(event_time_ms(fn, burst, warm=0))
    per = np.array(per)
    return {"seconds": round(time.perf_counter() - t0, 2), "launches": int(len(per) * burst),
            "solves_per_s": round(B / (per.mean() * 1e-3), 1), "ms_per_launch_mean": round(float(per.mean()), 4),
            "ms_per_launch_min_burst": round(float(per.min()), 4), "ms_per_launch_max_burst": round(float(per.max()), 4),
            "burst": burst}


def config3_leg(dev, reps: int) -> dict:
    """BASELINE config 3 (batch 4096, horizon N = 20, 10 iterations, one GPU): the fused step kernel
    (mpc_step_reg_kernel<20>: former + cold PDIPM, one launch) timed with HIP events on the launch
    stream, after the timed steps (steady clocks), and its FP64 roofline fraction (SURVEY 8d flops)."""
    wl = make_workload(C3_B, C3_N, seed=3000)
    inputs = [torch.from_numpy(x).to(dev) for x in wl.inputs]
    bufs = solver.MPCSolveBuffers.allocate(C3_N, C3_B, dev)
    ms = event_time_ms(lambda: solver.mpc_solve(inputs, C3_N, C3_K, 1.0, buffers=bufs), max(reps, 20), warm=3)
    flops = WORK[C3_N]["flops_per_iter"] * C3_K * C3_B
    idx = np.arange(0, C3_B, C3_B // C3_SAMPLE)
    return {"workload": f"batch {C3_B}, N={C3_N}, {C3_K} PDIPM iters, standing gait (BASELINE configs[2])",
            "kernel": solver_kernel_name(C3_N), "kernel_ms": round(ms, 4),
            "solves_per_s": round(C3_B / (ms * 1e-3), 1),
            "frac": round(flops / (ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, 6),
            "_wl": [x[idx] for x in wl.inputs], "_x": bufs.outputs[0][idx].cpu().numpy()}


def config3_parity(sample_inputs, x, threads: int) -> dict:
    """u0 of the config-3 sample (64 strided envs of the timed batch) vs the oracle (checker only)."""
    from oracle import oracle
    ref = oracle.mpc_solve(C3_N, C3_K, sample_inputs, y0=1.0, nthreads=threads)[0]
    ug, ur = x[:, 12 * C3_N:12 * C3_N + 12], ref[:, 12 * C3_N:12 * C3_N + 12]
    du = np.abs(ug - ur)
    return {"max_rel_du": float((du.max(axis=1) / np.abs(ur).max(axis=1)).max()),
            "max_rel_x": float((np.abs(x - ref).max(axis=1) / np.abs(ref).max(axis=1)).max()),
            "parity_envs": int(x.shape[0])}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus is not None and a.gpus > 1:
        sys.exit(launch_ranks(a, argv))  # this process only starts and joins the ranks
    _claim_stdout()
    world = int(env_world or "1")
    if a.gpus is None:  # torchrun --nproc-per-node N bench.py: the launcher's WORLD_SIZE decides
        a.gpus = world
    if a.gpus < 1 or world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world} ranks were launched", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    hook = os.environ.get("SRBD_BENCH_SOLVE_HOOK")
    # rehearsal hooks for the N > 1 path on a one-GPU box (never set by the driver): all ranks on
    # device 0, and gloo instead of RCCL (RCCL rejects two ranks on one device)
    one_device = os.environ.get("SRBD_BENCH_ONE_DEVICE") == "1"
    backend = "gloo" if hook else os.environ.get("SRBD_BENCH_BACKEND", "nccl")
    if one_device:
        local = 0
    if not hook and local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible", file=sys.stderr)
        sys.exit(2)
    if env_world is not None:  # under a launcher (ours or torch.distributed.run): a process group, even of one
        import torch.distributed as dist_mod
        dist = dist_mod
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()  # n_gpus = the ranks that joined
        rank = dist.get_rank()
    N, K, B = a.horizon, a.iters, a.batch_per_gpu
    d = Dims(N)
    if hook:
        return hook_main(a, hook, dist, world, rank, N, K, B, d)
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

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

    elapsed, u0_last, own_elapsed = run_timed(sh, inputs, a, dist, world, dev)
    ms_step = 1e3 * elapsed / a.steps
    value = world * B * a.steps / elapsed
    if rank == 0 and a.dump_u0:
        np.save(a.dump_u0, u0_last.cpu().numpy())

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
    dropin = None
    if rank == 0 and not a.no_dropin:
        dropin = dropin_leg(inputs, N, B, a.kernel_reps)
    ms_gather = None
    if dist is not None:
        u0 = bufs.outputs[0][:, 12 * N:12 * N + 12]
        ms_gather = event_time_ms(lambda: sh.gather_u0(u0), a.kernel_reps)
    ranks = rank_spread(dist, dev if backend == "nccl" else torch.device("cpu"), ms_fused,
                        ms_gather or 0.0, own_elapsed)
    sustained = None
    if a.sustain_seconds > 0:
        sustained = sustained_leg(lambda: solver.mpc_solve(inputs, N, K, 1.0, buffers=bufs), B, a.sustain_seconds)
    # BASELINE config 3 (batch 4096, N = 20, K = 10) under the driver's clock: its fused step kernel
    # timed with HIP events (+ a 64-env oracle parity sample in the CPU leg below)
    c3 = None
    if rank == 0 and (N, K) == (10, 10) and not a.no_config3:
        c3 = config3_leg(dev, a.kernel_reps)
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
        quota = _cgroup_cpu_quota()
        # thread scaling inside the process's CPU share (1 .. threads, ~1 s each): the evidence for
        # (or against) the linear per-core extrapolation to the whole host below
        scaling = {}
        t_ = 1
        while t_ <= threads:
            oracle.mpc_solve(N, K, sub, y0=1.0, nthreads=t_)
            ns, ts = 0, 0.0
            while ts < 1.0:
                t1 = time.perf_counter()
                oracle.mpc_solve(N, K, sub, y0=1.0, nthreads=t_)
                ts += time.perf_counter() - t1
                ns += sample
            scaling[str(t_)] = round(ns / ts, 1)
            t_ = t_ * 2 if t_ * 2 <= threads or t_ == threads else threads
        full = None
        if quota is not None and quota < affinity:
            # the CPU controller caps this process at `quota` CPUs whatever its affinity: a run with
            # every CPU of the affinity set would time the quota, not the host
            full = {"value": None, "reason": f"cgroup cpu.max allows {quota:g} CPUs of the {affinity} in the "
                                             f"affinity set: the whole host cannot be timed from this process"}
        if a.cpu_full_host and full is None:  # measured on every CPU of the affinity set (opt-in)
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
                        "full_host_measured": full, "cgroup_cpu_quota": quota,
                        "thread_scaling_solves_per_s": scaling},
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
        if c3 is not None:
            c3.update(config3_parity(c3.pop("_wl"), c3.pop("_x"), threads))
    if c3 is not None:
        c3.pop("_wl", None)
        c3.pop("_x", None)
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
                       # the register kernels' refinement mode (srbd_set_refinement)
                       "refinement": {0: "adaptive", 1: "every_iteration"}.get(_native.current_refinement(),
                                                                               "policy"),
                       "parallelism": f"dp{world}" + (f" (u0 all_gather over {'RCCL' if backend == 'nccl' else backend})"
                                                      if world > 1 else "")},
            # solves/s without the u0 gather (every rank's shard solve alone), N > 1 only
            "value_without_gather": (round(world * B / (ms_main * 1e-3), 1) if dist is not None else None),
            "kernels_ms": {"mpc_step_fused": round(ms_fused, 4) if fused else None,
                           "qp_former": round(ms_former, 4), "pdipm": round(ms_pdipm, 4),
                           "u0_all_gather": None if ms_gather is None else round(ms_gather, 4)},
            "build_id": _native.build_id(),  # source hash libsrbd_mpc.so was built from (build.py)
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
            "controller_step": ctrl,
            # the reference caller's own schedule through the CusADi-ABI drop-ins (INTEGRATION.md option A)
            "dropin_step_ms": None if dropin is None else dropin["literal_ms"],
            "dropin_step": dropin,
            "sustained": sustained,  # this rank's step kernel back to back for --sustain-seconds
            "config3": c3,  # BASELINE configs[2]: batch 4096, N = 20, 10 iterations, one GPU
            "ranks": ranks,  # N > 1: per-rank solve / gather / timed-region spread
        }
        emit(line)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
