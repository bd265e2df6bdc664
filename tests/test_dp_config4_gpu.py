"""BASELINE config 4 at its own shape (best_config.sh:4: RotatE FB15k-237,
E = 14541, R = 237, d = 1000 -de, γ = 9, b = 1024 per rank, n = 256, -adv):
the data-parallel exchanges run on cuda:0 with 2, 4 and 8 ranks (gloo; the
driver's 8-GPU runs use RCCL) for two fused-Adam steps (tail-, then head-
batch) and must equal ONE process training on the global batch of
world × 1024 rows bit for bit — at world 8 that is config 4's own global
batch of 8192 rows with the exchange `auto` picks there:

  * "owner" (forced at world 2 and 4): the row factors all-gathered, each rank's
    entity pass + fused Adam over its 1/N of the rows in OWNER_CHUNKS chunks,
    the chunks' rows all-gathered behind the next chunk's pass
    (partition.EntityRowPartition exchange "factors"; 14541 rows = 7271 + 7270
    at world 2, 3636 ×3 + 3633 at world 4, 1818 ×7 + 1815 at world 8, so the
    chunked all-gather, its slice rule and the owner's CSR range run at the
    real row counts);
  * "factors" (the world-2 default): the factors all-gathered, the global
    entity pass on every rank.

Bit-identity is checked on the whole entity and relation tables and on every
owner's Adam moments (sha256 of the bytes, so the 116 MB tables never cross a
process boundary), and the losses of both steps.  Then 8 rows' scores of the
trained rank-0 model are checked against the oracle's op chain on the trained
table (SURVEY §8c tolerance)."""
import hashlib
import os
import socket
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import score_tol, spawn_ranks
from knowledgegraphembedding_amd import KGEAdam, KGEModel, synth

pytestmark = pytest.mark.gpu

E, R, D, B, N, GAMMA, LR = 14541, 237, 1000, 1024, 256, 9.0, 5e-5
ROWS8 = [0, 1, 100, 511, 512, 777, 1000, 1023]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sha(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()


def _model():
    torch.manual_seed(0)
    return KGEModel("RotatE", E, R, D, GAMMA, True, False).to("cuda:0")


def _batches(world, dev):
    """The global batches of the two steps (world × B rows, rank order)."""
    out = []
    for k, mode in enumerate(("tail-batch", "head-batch")):
        pos, neg, w = synth.kge_batch(400 + k, world * B, N, E, R)
        out.append((torch.from_numpy(pos).to(dev), torch.from_numpy(neg).to(dev), torch.from_numpy(w).to(dev), mode))
    return out


def _args(group):
    return Namespace(cuda=True, negative_adversarial_sampling=True, adversarial_temperature=1.0, uni_weight=False,
                     regularization=0.0, dp_group=group, dp_exchange=None)


def _worker(rank, world, port, exchange, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _model()
    args = _args(dist.group.WORLD)
    if exchange == "owner":
        from knowledgegraphembedding_amd.partition import EntityRowPartition
        part = EntityRowPartition(model, dist.group.WORLD, exchange="factors")
        params = part.parameters()
    else:
        part = None
        args.dp_exchange = "factors"
        params = [p for p in model.parameters() if p.requires_grad]
    opt = KGEAdam(params, lr=LR)
    sl = slice(rank * B, (rank + 1) * B)
    it = iter([(p[sl], n[sl], w[sl], m) for p, n, w, m in _batches(world, "cuda:0")])
    logs = [dict(KGEModel.train_step(model, opt, it, args)) for _ in range(2)]
    torch.cuda.synchronize()
    res = {"logs": logs, "ent": _sha(model.entity_embedding), "rel": _sha(model.relation_embedding)}
    if part is not None:
        st = opt.state[part.shard]
        n_own = part.nown
        res.update(lo=min(part.lo, E), hi=min(part.lo, E) + n_own, m=_sha(st["exp_avg"][:n_own]),
                   v=_sha(st["exp_avg_sq"][:n_own]))
    else:
        st = opt.state[model.entity_embedding]
        res.update(lo=0, hi=E, m=_sha(st["exp_avg"]), v=_sha(st["exp_avg_sq"]))
    if rank == 0:  # the trained model's scores of 8 rows, for the oracle check
        pos, neg, _, _ = _batches(world, "cuda:0")[0]
        with torch.no_grad():
            res["scores8"] = model((pos[ROWS8], neg[ROWS8]), "tail-batch").cpu().numpy()
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange", [(2, "owner"), (4, "owner"), (8, "owner"), (2, "factors")])
def test_config4_shape_matches_one_process(world, exchange):
    out = mp.Manager().dict()
    spawn_ranks(_worker, (world, _free_port(), exchange, out), world)
    model = _model()
    opt = KGEAdam([p for p in model.parameters() if p.requires_grad], lr=LR)
    it = iter(_batches(world, "cuda:0"))
    ref_logs = [dict(KGEModel.train_step(model, opt, it, _args(None))) for _ in range(2)]
    torch.cuda.synchronize()
    st = opt.state[model.entity_embedding]
    ent_sha, rel_sha = _sha(model.entity_embedding), _sha(model.relation_embedding)
    covered = 0
    for rank in range(world):
        r = out[rank]
        assert r["ent"] == ent_sha, (world, exchange, rank, "entity table")
        assert r["rel"] == rel_sha, (world, exchange, rank, "relation table")
        lo, hi = r["lo"], r["hi"]
        assert r["m"] == _sha(st["exp_avg"][lo:hi]) and r["v"] == _sha(st["exp_avg_sq"][lo:hi]), (rank, lo, hi)
        covered += hi - lo
        for got, want in zip(r["logs"], ref_logs):
            for k in ("positive_sample_loss", "negative_sample_loss", "loss"):
                assert got[k] == want[k], (rank, k, got[k], want[k])
    assert covered == (E if exchange == "owner" else world * E)
    # oracle: the trained table's scores of 8 rows through the reference's op chain
    from oracle import kge_oracle as O
    pos, neg, _, _ = _batches(world, "cpu")[0]
    rng = model.embedding_range.item()
    ref = O.forward("RotatE", model.entity_embedding.detach().cpu(), model.relation_embedding.detach().cpu(), None,
                    (pos[ROWS8], neg[ROWS8]), "tail-batch", torch.Tensor([GAMMA]).item(), rng).numpy()
    got = out[0]["scores8"]
    assert np.all(np.abs(got - ref) <= score_tol(ref)), float(np.abs(got - ref).max())
