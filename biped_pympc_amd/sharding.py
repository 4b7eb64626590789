"""Data-parallel sharding of the batched SRBD-MPC step over GPUs.

Every environment is an independent QP, so the path partitions with no data-path collective: one
process per GPU solves a contiguous shard of the global batch (weak scaling). The one exchange is
the gather of the first-stage input u0 = x[12N : 12N + 12] of every env (96 B/env), which the
controller turns into joint torques for all robots (reference
``biped_pympc/convex_mpc/mpc_controller_cusadi.py:171-205`` reads u0 of every env). On MI355X the
gather is RCCL (backend "nccl") over xGMI; CPU tests run the same code over gloo.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch
import torch.distributed as dist


def shard_bounds(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) of ``total`` envs for ``rank`` of ``world`` (sizes differ by
    at most one; trailing ranks get empty shards when total < world)."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError(f"bad shard request total={total} world={world} rank={rank}")
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


class ShardedMPC:
    """One rank's share of a multi-GPU batched MPC solve.

    ``step(local_inputs)`` runs the fused former + PDIPM on this rank's shard and returns u0 of
    EVERY env of the global batch (``(total_envs, 12)``, global env order) on every rank.
    ``solve_fn(local_inputs) -> x`` may replace the HIP solve (tests run the CPU oracle through
    the same gather); by default it is ``solver.mpc_solve`` with preallocated buffers.
    """

    def __init__(self, N: int, n_iter: int, total_envs: int, device=None, y0: float = 1.0,
                 group=None, solve_fn: Callable[[Sequence[torch.Tensor]], torch.Tensor] | None = None):
        self.N, self.n_iter, self.total, self.y0, self.group = N, n_iter, total_envs, y0, group
        # with a process group the gather always runs through it, even at world size 1 (a one-GPU
        # job launched under torch.distributed exercises the same RCCL path as an 8-GPU one)
        self.collective = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.collective else 1
        self.rank = dist.get_rank(group) if self.collective else 0
        self.lo, self.hi = shard_bounds(total_envs, self.world, self.rank)
        self.sizes = [shard_bounds(total_envs, self.world, r) for r in range(self.world)]
        self.slot = max(h - l for l, h in self.sizes)  # padded per-rank block of the gather
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._solve_fn = solve_fn
        self._buffers = None
        self.x_local = None
        self.u0_all = torch.empty((total_envs, 12), dtype=torch.float64, device=self.device)
        self._ragged = any(h - l != self.slot for l, h in self.sizes)
        if self._ragged:
            self._send = torch.zeros((self.slot, 12), dtype=torch.float64, device=self.device)
            self._recv = torch.empty((self.world * self.slot, 12), dtype=torch.float64, device=self.device)
            keep = [r * self.slot + i for r, (l, h) in enumerate(self.sizes) for i in range(h - l)]
            self._keep = torch.tensor(keep, dtype=torch.int64, device=self.device)
        # step_async: double-buffered send / receive so a gather in flight never reads or writes a
        # buffer the next step is using
        self._abuf = None
        self._aidx = 0

    @property
    def local_envs(self) -> int:
        return self.hi - self.lo

    def local_slice(self, global_tensors: Sequence[torch.Tensor]) -> list[torch.Tensor]:
        """This rank's rows of batched ``(total_envs, ...)`` tensors (contiguous views)."""
        return [t[self.lo:self.hi] for t in global_tensors]

    def _solve(self, local_inputs) -> torch.Tensor:
        if self._solve_fn is not None:
            return self._solve_fn(local_inputs)
        from biped_pympc_amd import solver
        if self._buffers is None:
            self._buffers = solver.MPCSolveBuffers.allocate(self.N, self.local_envs, self.device)
        return solver.mpc_solve(list(local_inputs), self.N, self.n_iter, self.y0, self._buffers)[0]

    def step(self, local_inputs: Sequence[torch.Tensor]) -> torch.Tensor:
        if local_inputs[0].shape[0] != self.local_envs:
            raise ValueError(f"rank {self.rank}: expected {self.local_envs} envs, got {local_inputs[0].shape[0]}")
        self.x_local = self._solve(local_inputs)
        self.gather_u0(self.x_local[:, 12 * self.N:12 * self.N + 12])
        return self.u0_all

    def step_async(self, local_inputs: Sequence[torch.Tensor]) -> "PendingGather":
        """Like ``step`` but the u0 gather is left running on the collective's own stream (RCCL),
        so it overlaps the next step's solve; ``.wait()`` on the returned handle yields u0 of every
        env as a tensor of its own (later steps never overwrite it). Two steps' gathers may be in
        flight: the step after next waits for this one before reusing its send / receive pair
        (``PendingGather.wait`` is idempotent)."""
        if local_inputs[0].shape[0] != self.local_envs:
            raise ValueError(f"rank {self.rank}: expected {self.local_envs} envs, got {local_inputs[0].shape[0]}")
        self.x_local = self._solve(local_inputs)
        u0 = self.x_local[:, 12 * self.N:12 * self.N + 12]
        if not self.collective:  # the next solve reuses x_local: hand out a copy (96 B/env)
            return PendingGather(u0.clone(), None, None)
        if self._abuf is None:
            mk = lambda *sh: torch.zeros(sh, dtype=torch.float64, device=self.device)  # noqa: E731
            self._abuf = [(mk(self.slot, 12), mk(self.world * self.slot, 12)) for _ in range(2)]
            self._apending = [None, None]
        k = self._aidx
        self._aidx ^= 1
        if self._apending[k] is not None:  # the gather that used this buffer pair two steps ago
            self._apending[k].wait()
        send, recv = self._abuf[k]
        send[:self.local_envs].copy_(u0)  # on the compute stream, before the collective is enqueued
        if dist.get_backend(self.group) == "nccl":
            work = dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)
        else:
            work = dist.all_gather(list(recv.split(self.slot)), send, group=self.group, async_op=True)
        keep = self._keep if self._ragged else None
        self._apending[k] = PendingGather(recv, work, keep)
        return self._apending[k]

    @property
    def buffers(self):
        """The preallocated solver buffers of the default (HIP) solve, once a step has run."""
        return self._buffers

    def gather_u0(self, u0_local: torch.Tensor) -> torch.Tensor:
        """All-gather the shards' u0 into ``self.u0_all`` in global env order."""
        if not self.collective:
            self.u0_all = u0_local  # no process group: a view of the solution, no copy in the step
            return self.u0_all
        into_tensor = dist.get_backend(self.group) == "nccl"  # RCCL; gloo lacks the fused form
        if not self._ragged:
            if into_tensor:
                dist.all_gather_into_tensor(self.u0_all, u0_local.contiguous(), group=self.group)
            else:
                dist.all_gather(list(self.u0_all.split(self.slot)), u0_local.contiguous(), group=self.group)
            return self.u0_all
        self._send[:self.local_envs].copy_(u0_local)
        if into_tensor:
            dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
        else:
            dist.all_gather(list(self._recv.split(self.slot)), self._send, group=self.group)
        torch.index_select(self._recv, 0, self._keep, out=self.u0_all)
        return self.u0_all


class PendingGather:
    """Handle of an in-flight u0 gather (``ShardedMPC.step_async``)."""

    def __init__(self, buf: torch.Tensor, work, keep: torch.Tensor | None):
        self._buf, self._work, self._keep, self._out = buf, work, keep, None

    def wait(self) -> torch.Tensor:
        if self._out is None:
            if self._work is not None:
                self._work.wait()  # the current stream now waits for the collective
            # a copy: the receive buffer is reused by the gather two steps later
            self._out = self._buf.clone() if self._keep is None else self._buf.index_select(0, self._keep)
        return self._out
