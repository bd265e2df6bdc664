"""The chunked row exchange of the owner-computes step (partition.py
EntityRowPartition.put_chunk / gather, exchange "factors") with world 2 and 3
over gloo on CPU: every rank overwrites its own shard chunk by chunk, starts
each chunk's all-gather as soon as that chunk is written (as _owner_step does
after each chunk's entity pass), and after gather() every rank's replica must
hold every rank's rows — including the last shard's padding rows — exactly
where a single all-gather of the whole shards puts them.  The kernels' side
(bit-identical updates per chunk) is tests/test_dp_owner_gpu.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from knowledgegraphembedding_amd import KGEModel, partition

E, R, D = 301, 5, 8  # 151 / 101 owned rows at world 2 / 3: 4 / 3 chunks of ≥ 32 rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _owned(rank, rows, d2):
    """The values rank `rank` writes into its shard (a function of rank and row)."""
    r = torch.arange(rows, dtype=torch.float32)[:, None]
    c = torch.arange(d2, dtype=torch.float32)[None, :]
    return 1000.0 * (rank + 1) + 10.0 * r + c * 0.5


def _worker(rank, world, port, chunks, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = KGEModel("RotatE", E, R, D, 12.0, True, False)
    partition.OWNER_CHUNKS = chunks
    part = partition.EntityRowPartition(model, dist.group.WORLD, exchange="factors")
    vals = _owned(rank, part.rows, part.dim)
    spans = part._owner_chunks()
    for c0, c1 in spans:
        with torch.no_grad():
            part.full[part.lo + c0:part.lo + c1].copy_(vals[c0:c1])  # the owner's in-place update of chunk c
        part.put_chunk(c0, c1)
    part.gather()
    out[rank] = {"full": part.full.clone(), "spans": spans, "rows": part.rows,
                 "ent": model.entity_embedding.detach().clone()}
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 1), (2, 4), (3, 3)])
def test_chunked_row_gather_places_every_shard(world, chunks):
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), chunks, out), nprocs=world, join=True)
    rows = out[0]["rows"]
    want = torch.cat([_owned(r, rows, 2 * D) for r in range(world)])
    assert len(out[0]["spans"]) == max(1, min(chunks, rows // 32)) == chunks
    for r in range(world):
        assert torch.equal(out[r]["full"], want), r
        assert torch.equal(out[r]["ent"], want[:E]), r  # the model's table views the replica
