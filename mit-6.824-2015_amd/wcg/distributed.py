"""Multi-GPU word count: one process per GPU, the ihash shuffle as an RCCL all-to-all-v.

Reference semantics being distributed (paths relative to /root/reference):
  * DoMap partitions every key by ihash(key) % nReduce (src/mapreduce/mapreduce.go:214-223);
  * DoReduce r gathers partition r from every map output (mapreduce.go:242-263);
  * Merge reads every -res-r and sorts all keys (mapreduce.go:284-321).
Here each rank maps a line-aligned byte range (rank = a group of map jobs), pre-aggregates
(key, count) on its GPU, exports its records bucketed by owner = (ihash % nReduce) % world
(partition r is owned by rank r % world), and one all_to_all_single (RCCL grouped
send/recv over xGMI) delivers every partition to its owner, which reduces it (= DoReduce for
its partitions).  The final Merge gathers the owners' disjoint results on rank 0.

The module is device-agnostic: it only needs an engine with export_tensor/import_tensor/
reset/reduce/result, so the CPU tests drive it with the `gloo` backend and an oracle-backed
stand-in engine (tests/test_distributed.py); the product engine is wcg.Engine.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

RECORD_BYTES = 32


# ---------------------------------------------------------------- device copies (HIP runtime)
_hip = None


def _hiprt():
    global _hip
    if _hip is None:
        for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _hip is None:
            raise ImportError("libamdhip64.so not found")
        _hip.hipMemcpyAsync.restype = ctypes.c_int
        _hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                       ctypes.c_void_p]
    return _hip


def device_copy(dst: int, src: int, nbytes: int, stream: int = 0) -> None:
    """hipMemcpyAsync device-to-device on `stream` (plumbing between libwcg and torch buffers)."""
    if nbytes == 0:
        return
    rc = _hiprt().hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3, ctypes.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed: {rc}")


# ---------------------------------------------------------------- range partitioning
def line_aligned_ranges(total: int, world: int, byte_at) -> List[Tuple[int, int]]:
    """Cut [0, total) into `world` ranges at positions just after a '\\n' (Split's cut points,
    mapreduce.go:166-172).  byte_at(i) returns the input byte at i.  Any cut after an ASCII
    non-letter is safe: no rune and no token can straddle it."""
    cuts = [0]
    for r in range(1, world):
        p = max(cuts[-1], (total * r) // world)
        while p < total and byte_at(p - 1) != 0x0A:
            p += 1
        cuts.append(p)
    cuts.append(total)
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


# ---------------------------------------------------------------- the shuffle
def _exchange(send: torch.Tensor, send_units: List[int], group=None) -> Tuple[torch.Tensor, List[int]]:
    """all-to-all-v of 32-byte record units.  Counts first (small all_to_all), then payload."""
    world = dist.get_world_size(group)
    dev = send.device
    sc = torch.tensor(send_units, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv_units = [int(x) for x in rc.tolist()]
    recv = torch.empty(max(sum(recv_units), 1) * RECORD_BYTES, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv[: sum(recv_units) * RECORD_BYTES], send[: sum(send_units) * RECORD_BYTES],
                           output_split_sizes=[u * RECORD_BYTES for u in recv_units],
                           input_split_sizes=[u * RECORD_BYTES for u in send_units], group=group)
    return recv, recv_units


def shuffle(engine, nreduce: int, group=None) -> None:
    """The ihash shuffle: export the local aggregate by owner, all-to-all it, and import what
    this rank owns.  Afterwards `engine` holds exactly the (aggregated) keys of the partitions
    this rank owns (mapreduce.go:214-223 partitioning, :242-263 gathering)."""
    world = dist.get_world_size(group)
    send, units = engine.export_tensor(nreduce, world)
    recv, rcv_units = _exchange(send, units, group)
    engine.reset()
    engine.import_tensor(recv, sum(rcv_units))


def shuffle_reduce(engine, nreduce: int, group=None) -> int:
    """shuffle(), then DoReduce for the owned partitions (sorted and formatted on this rank).
    Returns the number of keys this rank owns."""
    shuffle(engine, nreduce, group)
    nkeys, _ = engine.reduce()
    return nkeys


def gather_merge(engine, root_engine, root: int = 0, group=None, fetch: bool = True) -> Optional[bytes]:
    """Merge (mapreduce.go:284-321) across ranks: every owner sends its keys to `root`, whose
    engine re-sorts the union (the owners' key sets are disjoint).  Returns the merged file
    bytes on root (fetch=False: leaves them in root_engine's device buffer and returns b""),
    None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    send, units = engine.export_tensor(1, 1)
    n = units[0]
    sizes = [0] * world
    sizes[root] = n
    recv, rcv_units = _exchange(send, sizes, group)
    if rank != root:
        return None
    root_engine.reset()
    root_engine.import_tensor(recv, sum(rcv_units))
    root_engine.reduce()
    return root_engine.result() if fetch else b""


class TorchEngine:
    """wcg.Engine + torch buffers for the collectives (device memory stays in HBM).

    host_staging=True hands the collectives host tensors instead (for the gloo backend, e.g.
    several ranks sharing one GPU in a test; RCCL needs one GPU per rank)."""

    def __init__(self, engine, stream_ptr: int = 0, host_staging: bool = False):
        self.e = engine
        self.stream = stream_ptr
        self.host_staging = host_staging

    def reset(self):
        self.e.reset()

    def reduce(self):
        return self.e.reduce()

    def result(self):
        return self.e.result()

    def export_tensor(self, nreduce: int, nranks: int):
        ptr, counts = self.e.export(nreduce, nranks)
        total = sum(counts)
        t = torch.empty(max(total, 1) * RECORD_BYTES, dtype=torch.uint8, device="cuda")
        device_copy(t.data_ptr(), ptr, total * RECORD_BYTES, self.stream)
        torch.cuda.current_stream().synchronize()
        return (t.cpu() if self.host_staging else t), counts

    def import_tensor(self, t: torch.Tensor, nunits: int):
        if not t.is_cuda:
            t = t.to("cuda")
        torch.cuda.current_stream().synchronize()
        self.e.import_records(t.data_ptr(), nunits)
        torch.cuda.current_stream().synchronize()     # t may be freed on return
