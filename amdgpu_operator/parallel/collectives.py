"""RCCL collective sweep: correctness + algBW/busBW across message sizes.

SURVEY.md §2.E lists a bench ``allreduce_sweep`` (8 B ... 1 GiB, all-reduce,
plus all-gather / reduce-scatter as a topology sanity check) next to the
validator's fixed-size check.  The reference has no collective at all
(/root/reference/README.md:1-220 runs only ``nvidia-smi``); this is the
MI355X-native measurement behind the "all-reduce busBW" row of BASELINE.md.

One process per GPU under ``torch.distributed.run`` (backend ``nccl`` is RCCL
on ROCm; ranks talk over xGMI).  The same code runs on CPU with ``gloo`` so the
multi-rank logic is testable without a GPU.  Every size is checked exactly
(rank r contributes r + 1, so every result is a small integer) before it is
timed; the reported time is the MAX over ranks (a collective is as slow as its
slowest rank).  busBW uses the rccl-tests factors: all-reduce 2(n-1)/n,
all-gather / reduce-scatter (n-1)/n, of the bytes of the full (gathered /
unscattered) tensor.
"""

from __future__ import annotations

import time
from dataclasses import asdict, dataclass

OPS = ("allreduce", "allgather", "reducescatter")

_BUS_FACTOR = {
    "allreduce": lambda n: 2.0 * (n - 1) / n,
    "allgather": lambda n: (n - 1) / n,
    "reducescatter": lambda n: (n - 1) / n,
}


@dataclass
class SweepRow:
    op: str
    dtype: str
    bytes: int
    world: int
    ms: float
    algbw_gbps: float
    busbw_gbps: float
    ok: bool


def default_sizes(min_bytes: int = 8, max_bytes: int = 1 << 30, factor: int = 4) -> list[int]:
    out, b = [], min_bytes
    while b <= max_bytes:
        out.append(b)
        b *= factor
    if out and out[-1] != max_bytes and max_bytes > min_bytes:
        out.append(max_bytes)
    return out


class _Clock:
    """CUDA events on a GPU, perf_counter + barrier on CPU (gloo)."""

    def __init__(self, torch, dist, group, cuda: bool):
        self.torch, self.dist, self.group, self.cuda = torch, dist, group, cuda

    def time_ms(self, fn, iters: int) -> float:
        torch = self.torch
        if self.cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / iters
        self.dist.barrier(group=self.group)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) * 1e3 / iters


def _elem_count(nbytes: int, esize: int, world: int) -> int:
    # a multiple of world elements, at least world
    n = max(world, nbytes // esize)
    return (n // world) * world


def run_op(op: str, nbytes: int, dtype, device, group=None, iters: int = 10, warmup: int = 2) -> SweepRow:
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    esize = torch.empty((), dtype=dtype).element_size()
    n = _elem_count(nbytes, esize, world)
    per = n // world
    expect = world * (world + 1) / 2.0
    full = torch.empty(n, device=device, dtype=dtype)
    part = torch.empty(per, device=device, dtype=dtype)

    if op == "allreduce":
        def launch():
            dist.all_reduce(full, group=group)

        full.fill_(rank + 1)
        launch()
        ok = bool(torch.all(full == expect).item())
    elif op == "allgather":
        def launch():
            dist.all_gather_into_tensor(full, part, group=group)

        part.fill_(rank + 1)
        launch()
        want = torch.arange(world, device=device, dtype=torch.float32).repeat_interleave(per) + 1
        ok = bool(torch.equal(full.float(), want))
    elif op == "reducescatter":
        def launch():
            dist.reduce_scatter_tensor(part, full, group=group)

        full.fill_(rank + 1)
        launch()
        ok = bool(torch.all(part == expect).item())
    else:
        raise ValueError(f"unknown collective {op!r}")

    cuda = full.is_cuda
    clock = _Clock(torch, dist, group, cuda)
    if op == "allreduce":
        full.fill_(1)  # keep repeated sums finite and exact
    for _ in range(warmup):
        launch()
    ms = clock.time_ms(launch, iters)
    t = torch.tensor([ms], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    ms = float(t.item())
    # all ranks agree on correctness
    okt = torch.tensor([0 if ok else 1], dtype=torch.int32, device=device)
    dist.all_reduce(okt, op=dist.ReduceOp.MAX, group=group)
    ok = okt.item() == 0
    total = n * esize
    algbw = total / (ms * 1e-3) / 1e9
    bus = algbw * _BUS_FACTOR[op](world) if world > 1 else 0.0
    return SweepRow(op, str(dtype).replace("torch.", ""), total, world, ms, algbw, bus, ok)


def sweep(sizes: list[int], ops=OPS, dtype=None, device=None, group=None, iters: int = 10,
          warmup: int = 2) -> list[SweepRow]:
    import torch

    dtype = dtype or torch.float32
    rows = []
    for op in ops:
        for b in sizes:
            # shorter loops for the big messages keep a 1 GiB sweep within seconds
            it = iters if b < (64 << 20) else max(2, iters // 4)
            rows.append(run_op(op, b, dtype, device, group, it, warmup))
    return rows


def rows_as_dicts(rows: list[SweepRow]) -> list[dict]:
    return [asdict(r) for r in rows]


def format_table(rows: list[SweepRow]) -> str:
    lines = [f"{'op':<14}{'dtype':<10}{'bytes':>12}{'ms':>10}{'algBW GB/s':>12}{'busBW GB/s':>12}  ok"]
    for r in rows:
        lines.append(f"{r.op:<14}{r.dtype:<10}{r.bytes:>12}{r.ms:>10.4f}{r.algbw_gbps:>12.1f}{r.busbw_gbps:>12.1f}  "
                     f"{'yes' if r.ok else 'NO'}")
    return "\n".join(lines)
