import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkge_hip.so)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_info():
    with open(GOLDEN / "golden.json") as f:
        return json.load(f)


def load_npz(name):
    return np.load(GOLDEN / name, allow_pickle=False)


@pytest.fixture(scope="session")
def g_scores():
    return load_npz("scores.npz")


@pytest.fixture(scope="session")
def g_train():
    return load_npz("train.npz")


@pytest.fixture(scope="session")
def g_ranks():
    return load_npz("ranks.npz")


@pytest.fixture(scope="session")
def g_sampler():
    return load_npz("sampler.npz")


@pytest.fixture(scope="session")
def g_countries():
    return load_npz("countries.npz")


MODEL_DIMS = {"TransE": (False, False), "DistMult": (False, False), "ComplEx": (True, True),
              "RotatE": (True, False), "pRotatE": (False, False)}


def dims(name, d):
    de, dr = MODEL_DIMS[name]
    return (2 * d if de else d), (2 * d if dr else d)


def erange_of(gamma, d):
    import torch
    return torch.Tensor([(torch.Tensor([gamma]).item() + 2.0) / d]).item()


def synth_tables(name, E, R, d, gamma, seed):
    from knowledgegraphembedding_amd import synth
    le, lr = dims(name, d)
    rng = erange_of(gamma, d)
    ent, rel = synth.kge_tables(seed, E, R, le, lr, rng)
    mod = np.array([[0.5 * rng]], dtype=np.float32) if name == "pRotatE" else None
    return ent, rel, mod, rng


def spawn_ranks(fn, args, nprocs):
    """mp.spawn for ranks that share ONE GPU (the -m gpu multi-rank tests):
    each rank limited to one HIP hardware queue.  With the default four per
    process, five processes on one card (the pytest parent holds its own)
    oversubscribe the card's hardware queue slots and the scheduler
    time-slices them: the world-4 query-shipping case took 138 s instead of
    5.4 s.  Product runs use one process per GPU."""
    import torch.multiprocessing as mp
    old = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = "1"  # inherited by the spawned ranks only (read at their HIP init)
    try:
        mp.spawn(fn, args=args, nprocs=nprocs, join=True)
    finally:
        if old is None:
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = old


def score_tol(ref):
    """|Δ| ≤ 1e-4 · max(|s_ref|, 1) — the north-star fp32 score tolerance."""
    return 1e-4 * np.maximum(np.abs(ref), 1.0)
