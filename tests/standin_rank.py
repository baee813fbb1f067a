"""One rank of the multi-GPU word count on the CPU, for the launcher tests (test infrastructure):
the N > 1 orchestration of bench.py (line-aligned ranges, shuffle, owners' DoReduce, Merge of the
runs at rank 0; wcg/distributed.py) over gloo with the oracle-backed stand-in engine of
tests/test_distributed.py.  Rank 0 prints one JSON line, as bench.py does.

  python -m torch.distributed.run ... tests/standin_rank.py [--fail-rank R] [--hang-rank R]
                                      [--ignore-term-rank R] [--pid-dir D]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mit-6.824-2015_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fail-rank", type=int, default=-1)
    ap.add_argument("--hang-rank", type=int, default=-1)
    ap.add_argument("--ignore-term-rank", type=int, default=-1,
                    help="this rank ignores SIGTERM and hangs (only SIGKILL ends it)")
    ap.add_argument("--pid-dir", default=None, help="each rank writes its pid here")
    ap.add_argument("--nreduce", type=int, default=64)
    args = ap.parse_args()
    import torch.distributed as dist
    from tests.test_distributed import OracleEngine, corpus
    from tests.oracle_bridge import wc_ref
    from wcg import distributed as wd
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if args.pid_dir:
        with open(os.path.join(args.pid_dir, f"rank{rank}.pid"), "w") as f:
            f.write(str(os.getpid()))
    if rank == args.ignore_term_rank:
        import signal
        signal.signal(signal.SIGTERM, signal.SIG_IGN)
        time.sleep(3600)
    dist.init_process_group("gloo")
    if rank == args.fail_rank:
        raise SystemExit(7)
    if rank == args.hang_rank:
        time.sleep(3600)
    data = corpus()
    lo, hi = wd.line_aligned_ranges(len(data), world, lambda i: data[i])[rank]
    eng = OracleEngine()
    eng.map_bytes(data[lo:hi])
    wd.shuffle_reduce(eng, args.nreduce)
    merged = wd.gather_merge(eng)
    if rank == 0:
        ok = merged == wc_ref.merged_output(wc_ref.word_count(data))
        print(json.dumps({"n_gpus": world, "verified_vs_oracle": ok, "bytes": len(data)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
