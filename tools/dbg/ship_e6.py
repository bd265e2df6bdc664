"""Diagnostic: where the query-shipping GPU test's e=6 / world-4 case spends
its time (tests/test_ship_gpu.py, RotatE, shards of 2 rows, the last empty).
Each rank dumps its Python stack every 20 s and prints per-step wall times."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import test_ship_gpu as T  # noqa: E402
from knowledgegraphembedding_amd import KGEAdam, KGEModel  # noqa: E402


def worker(rank, world, port, e):
    faulthandler.dump_traceback_later(20, repeat=True, file=sys.stderr)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from knowledgegraphembedding_amd.partition import EntityRowPartition
    model = T._model("RotatE", e, T.D)
    part = EntityRowPartition(model, dist.group.WORLD, exchange="queries")
    opt = KGEAdam(part.parameters(), lr=T.LR)
    print(f"rank {rank} setup {time.perf_counter() - t0:.2f}s nown={part.nown} lo={part.lo}", flush=True)
    sl = slice(rank * T.B // world, (rank + 1) * T.B // world)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in T._batches("cuda:0", e)])
    for s in range(T.STEPS):
        t1 = time.perf_counter()
        log = dict(KGEModel.train_step(model, opt, it, T._args(dist.group.WORLD, 0.0, False)))
        torch.cuda.synchronize()
        print(f"rank {rank} step {s} {time.perf_counter() - t1:.2f}s loss {log['loss']:.6f}", flush=True)
    t1 = time.perf_counter()
    part.materialize()
    torch.cuda.synchronize()
    print(f"rank {rank} materialize {time.perf_counter() - t1:.2f}s", flush=True)
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def test_worker(rank, world, port, e, out):
    """The GPU test's own worker (T._worker), with a stack dump every 20 s."""
    faulthandler.dump_traceback_later(20, repeat=True, file=sys.stderr)
    t0 = time.perf_counter()
    T._worker(rank, world, port, "RotatE", 0.0, False, e, T.D, {}, out)
    print(f"rank {rank} test worker {time.perf_counter() - t0:.2f}s", flush=True)
    faulthandler.cancel_dump_traceback_later()


def run_as_test(world=4, e=6):
    torch.ones(4, device="cuda:0").sum().item()  # the pytest parent holds a HIP context too
    t0 = time.perf_counter()
    out = mp.Manager().dict()
    mp.spawn(test_worker, args=(world, T._free_port(), e, out), nprocs=world, join=True)
    print(f"spawn as in the test: {time.perf_counter() - t0:.2f}s", flush=True)


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    e = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    if len(sys.argv) > 3 and sys.argv[3] == "test":
        run_as_test(world, e)
    else:
        mp.spawn(worker, args=(world, T._free_port(), e), nprocs=world, join=True)
    print("done", flush=True)
