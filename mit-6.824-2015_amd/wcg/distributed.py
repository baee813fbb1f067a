"""Multi-GPU word count: one process per GPU, the ihash shuffle as an RCCL all-to-all-v.

Reference semantics being distributed (paths relative to /root/reference):
  * DoMap partitions every key by ihash(key) % nReduce (src/mapreduce/mapreduce.go:214-223);
  * DoReduce r gathers partition r from every map output (mapreduce.go:242-263);
  * Merge reads every -res-r and sorts all keys (mapreduce.go:284-321).
Here each rank maps a line-aligned byte range (rank = a group of map jobs), pre-aggregates
(key, count) on its GPU, exports its records bucketed by owner = (ihash % nReduce) % world
(partition r is owned by rank r % world), and the exchange delivers every partition to its
owner, which reduces it (= DoReduce for its partitions: sort + format).  The final Merge sends
the owners' sorted runs to rank 0, which merges them on its GPU (k-way, by pairwise merge
passes).

Two transports carry the exchange and the gather:
  * the product path (bench.py with backend nccl, after init_comm()): both run inside libwcg -
    wcg_exchange = ncclAllGather of every rank's status and per-owner record counts, then ONE
    ncclGroupStart/End of ncclSend/ncclRecv pairs (all-to-all-v over xGMI, each rank's records
    straight from its export buffer into the owners' import buffers), and wcg_gather_merge =
    grouped ncclSend/ncclRecv of the sorted runs to rank 0 and its k-way merge;
  * the portable path (gloo: CPU tests, host-staged rehearsals on one GPU): _exchange() below,
    torch.distributed all_to_all_single of the counts, then of the records.

The module is device-agnostic: it only needs an engine with export_tensor/import_tensor/reset/
reduce/result/result_tensor/merge_runs_tensor, so the CPU tests drive it with the `gloo` backend
and an oracle-backed stand-in engine (tests/test_distributed.py); the product engine is
wcg.Engine wrapped in TorchEngine.
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
def _exchange(send: torch.Tensor, send_units: List[int], group=None, unit: int = RECORD_BYTES
              ) -> Tuple[torch.Tensor, List[int]]:
    """all-to-all-v of `unit`-byte items.  Counts first (small all_to_all), then payload."""
    world = dist.get_world_size(group)
    dev = send.device
    sc = torch.tensor(send_units, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv_units = [int(x) for x in rc.tolist()]
    recv = torch.empty(max(sum(recv_units), 1) * unit, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv[: sum(recv_units) * unit], send[: sum(send_units) * unit],
                           output_split_sizes=[u * unit for u in recv_units],
                           input_split_sizes=[u * unit for u in send_units], group=group)
    return recv, recv_units


def init_comm(engine, group=None) -> None:
    """Give the library its own RCCL communicator (wcg_comm_init): rank 0 makes the unique id,
    torch.distributed hands it to every rank (the reference's config-5 master would carry it in
    its RPC).  After this, shuffle() and gather_merge() run inside libwcg (wcg_exchange,
    wcg_gather_merge) instead of through torch collectives."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    e = engine.e if isinstance(engine, TorchEngine) else engine
    obj = [e.comm_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    e.comm_init(obj[0], rank, world)
    if isinstance(engine, TorchEngine):
        engine.in_library = True


def shuffle(engine, nreduce: int, group=None) -> None:
    """The ihash shuffle: export the local aggregate by owner straight into the send buffer,
    all-to-all it, and import what this rank owns.  Afterwards `engine` holds exactly the
    (aggregated) keys of the partitions this rank owns (mapreduce.go:214-223 partitioning,
    :242-263 gathering).  With init_comm() done this is one wcg_exchange call (RCCL inside the
    library, one host read of the unit counts)."""
    if getattr(engine, "in_library", False):
        engine.e.exchange(nreduce)
        return
    world = dist.get_world_size(group)
    send, units = engine.export_tensor(nreduce, world)
    recv, rcv_units = _exchange(send, units, group)
    engine.reset()
    engine.import_tensor(recv, sum(rcv_units))


def shuffle_reduce(engine, nreduce: int, group=None) -> int:
    """shuffle(), then DoReduce for the owned partitions: this rank sorts and formats its keys
    (its sorted run of the final Merge).  Returns the number of keys this rank owns."""
    shuffle(engine, nreduce, group)
    nkeys, _ = engine.reduce()
    return nkeys


def gather_merge(engine, root: int = 0, group=None, fetch: bool = True) -> Optional[bytes]:
    """Merge (mapreduce.go:284-321) across ranks, after shuffle_reduce: every owner sends its
    sorted run (its formatted "key: count\n" output; the owners' key sets are disjoint) to
    `root`, which merges the runs on its GPU (wcg_merge_runs: ceil(log2 world) merge passes, no
    re-sort).  Returns the merged file bytes on root (fetch=False: leaves them in the root
    engine's device buffer and returns b""), None elsewhere."""
    if getattr(engine, "in_library", False):         # wcg_gather_merge: RCCL inside the library
        engine.e.gather_merge(root)
        if dist.get_rank(group) != root:
            return None
        return engine.result() if fetch else b""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    send, nbytes = engine.result_tensor()
    sizes = [0] * world
    sizes[root] = nbytes
    recv, run_bytes = _exchange(send, sizes, group, unit=1)
    if rank != root:
        return None
    engine.merge_runs_tensor(recv, run_bytes)
    return engine.result() if fetch else b""


class TorchEngine:
    """wcg.Engine + torch buffers for the collectives (device memory stays in HBM).

    The engine is bound to torch's current stream (when that is not the legacy default stream),
    so the export kernels, the collectives and the import kernels are ordered on one stream with
    no host waits between them.  On the default stream the engine keeps its own stream and every
    hand-over synchronises instead.  host_staging=True hands the collectives host tensors (for
    the gloo backend, e.g. several ranks sharing one GPU in a test; RCCL needs one GPU per rank).
    """

    def __init__(self, engine, stream_ptr: Optional[int] = None, host_staging: bool = False):
        self.e = engine
        self.host_staging = host_staging
        self.in_library = False                   # init_comm(): wcg_exchange / wcg_gather_merge
        cur = torch.cuda.current_stream().cuda_stream
        if stream_ptr is None:
            stream_ptr = cur
        if stream_ptr:
            engine.set_stream(stream_ptr)
        self.ordered = bool(stream_ptr) and stream_ptr == cur

    def reset(self):
        self.e.reset()

    def reduce(self):
        return self.e.reduce()

    def result(self):
        return self.e.result()

    def _before_engine(self):            # torch's writes (copies, collectives) land first
        if not self.ordered:
            torch.cuda.current_stream().synchronize()

    def _after_engine(self):             # the engine's writes / reads of a torch buffer are done
        if not self.ordered:
            self.e.sync()

    def export_tensor(self, nreduce: int, nranks: int):
        counts = self.e.export_count(nreduce, nranks)
        total = sum(counts)
        t = torch.empty(max(total, 1) * RECORD_BYTES, dtype=torch.uint8, device="cuda")
        self._before_engine()
        self.e.export_write(t.data_ptr())          # the send buffer itself: no extra copy
        self._after_engine()
        return (t.cpu() if self.host_staging else t), counts

    def import_tensor(self, t: torch.Tensor, nunits: int):
        if not t.is_cuda:
            t = t.to("cuda")
        self._before_engine()
        self.e.import_records(t.data_ptr(), nunits)
        self._after_engine()                     # ordered: t's memory is reused only after the import

    def result_tensor(self):
        """This rank's formatted output as a tensor (one device copy of at most a few MB per
        rank at the configs' vocabularies)."""
        _, nb = self.e.result_device()
        t = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
        self._before_engine()
        self.e.result_copy_device(t.data_ptr())
        self._after_engine()
        return (t.cpu() if self.host_staging else t), nb

    def merge_runs_tensor(self, t: torch.Tensor, run_bytes: List[int]):
        if not t.is_cuda:
            t = t.to("cuda")
        self._before_engine()
        return self.e.merge_runs(t.data_ptr(), run_bytes)     # synchronous
