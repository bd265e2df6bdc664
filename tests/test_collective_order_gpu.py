"""Stream ordering of gloo's async collectives on CUDA tensors (VERDICT r05
#1): does an async ``all_gather_into_tensor`` of CUDA tensors under gloo
(1) read its input only after the work queued before it on the caller's
stream, and (2) finish writing its output before the caller's stream runs
the first kernel queued after ``work.wait()``?

Each phase is arranged so that a missing dependency fails every time, not
by chance:

* input side — the caller's stream spins ~50 ms (``torch.cuda._sleep``),
  THEN fills the input; the collective is issued right after, from the host,
  while the spin still runs.  An input copy that does not wait for the
  caller's stream copies the old zeros;
* output side — the output is pre-filled with NaN on the caller's stream,
  the gathered buffer is 64 MB per rank (its host→device copy takes
  milliseconds), and a device comparison is queued immediately after
  ``wait()``.  A wait that does not order the caller's stream behind that
  copy compares against NaNs;
* the owner step's pattern (partition.put_chunk / gather): 4 chunk gathers
  of a replica's own rows in flight at once into per-chunk staging buffers
  reused across 3 steps, each put preceded by a spin, then wait + strided
  copy into the replica rows, then a device comparison; the values change
  every step, so a stale staging buffer shows as well as a zero one.

The ranks share cuda:0 (gloo between them), as every multi-rank GPU test
does.  The result decides whether the owner step's gloo path may rely on
gloo's own CUDA streams."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import spawn_ranks

pytestmark = pytest.mark.gpu

SPIN = 100_000_000  # torch.cuda._sleep cycles (tens of ms)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    vals = torch.arange(1, world + 1, device=dev, dtype=torch.float32).view(world, 1)

    # (1) input side
    n = 1 << 20
    x = torch.zeros(n, device=dev)
    o = torch.zeros(world * n, device=dev)
    torch.cuda.synchronize()
    torch.cuda._sleep(SPIN)
    x.fill_(rank + 1.0)
    w = dist.all_gather_into_tensor(o, x, async_op=True)
    w.wait()
    res["input_bad"] = int((o.view(world, n) != vals).sum().item())

    # (2) output side
    n = 16 << 20  # 64 MB per rank
    x = torch.full((n,), rank + 1.0, device=dev)
    o = torch.full((world * n,), float("nan"), device=dev)
    w = dist.all_gather_into_tensor(o, x, async_op=True)
    w.wait()
    res["output_bad"] = int((o.view(world, n) != vals).sum().item())

    # (3) the owner step's chunked row gathers
    S, d, chunks = 4096, 256, 4
    full = torch.zeros(world * S, d, device=dev)
    stage = {}
    col = torch.arange(d, device=dev, dtype=torch.float32)
    rows = torch.arange(world * S, device=dev, dtype=torch.float32).view(-1, 1)
    step_rows = S // chunks
    bad = zero = 0
    for it in range(3):
        pending = []
        torch.cuda._sleep(SPIN // 4)
        full[rank * S:(rank + 1) * S] = (rows[rank * S:(rank + 1) * S] * 1000 + col + it * 0.5)
        for c0 in range(0, S, step_rows):
            c1 = c0 + step_rows
            st = stage.get(c0)
            if st is None:
                st = stage[c0] = torch.empty(world * (c1 - c0), d, device=dev)
            torch.cuda._sleep(SPIN // 16)  # the next chunk's entity pass
            pending.append((dist.all_gather_into_tensor(st, full[rank * S + c0:rank * S + c1], async_op=True),
                            st, c0, c1))
        for work, st, c0, c1 in pending:
            work.wait()
            full.view(world, S, d)[:, c0:c1].copy_(st.view(world, c1 - c0, d))
        want = rows * 1000 + col + it * 0.5
        diff = full != want
        bad += int(diff.any(1).sum().item())
        zero += int((full == 0).all(1).sum().item())
    res["owner_bad_rows"], res["owner_zero_rows"] = bad, zero
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_async_all_gather_stream_order(world):
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), out), world)
    got = {r: dict(out[r]) for r in range(world)}
    print("gloo ordering per rank:", got)
    for r, res in got.items():
        assert res == {"input_bad": 0, "output_bad": 0, "owner_bad_rows": 0, "owner_zero_rows": 0}, (r, res)
