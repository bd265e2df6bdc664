"""The C-ABI library loads and exports every symbol include/kge_hip.h declares;
host-side argument checks behave (no device work is launched here)."""
import ctypes as C
import re

import pytest

from conftest import REPO
from knowledgegraphembedding_amd import _lib


def _declared():
    text = (REPO / "include" / "kge_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kge_[a-z_0-9]+)\s*\(", text)))


def test_header_matches_binding_table():
    assert _declared() == sorted(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.kge_version()


def _desc(model=3, le=16, lr=8, ne=10, nr=3):
    d = _lib.ModelDesc()
    d.model, d.entity_dim, d.relation_dim, d.nentity, d.nrelation = model, le, lr, ne, nr
    d.gamma, d.phase_divisor, d.phase_divisor_p = 12.0, 0.1, 0.1
    buf = (C.c_float * 64)()
    d.entity_embedding = C.cast(buf, C.c_void_p).value
    d.relation_embedding = C.cast(buf, C.c_void_p).value
    d.modulus = C.cast(buf, C.c_void_p).value
    return d, buf


@pytest.mark.parametrize("model,le,lr,status", [
    (7, 16, 16, 1),    # unknown model → ValueError('model %s not supported'), model.py:64
    (3, 16, 16, 3),    # RotatE needs -de and not -dr, model.py:66-67
    (2, 16, 8, 3),     # ComplEx needs -de and -dr, model.py:69-70
    (0, 16, 8, 3),     # TransE rows must broadcast
    (1, 8192, 8192, 6),  # beyond the compiled row range
    (1, 2049, 2049, 6),  # (half-)rows up to 2048 floats, any alignment (2049: one past)
    (3, 4098, 2049, 6),
])
def test_model_validation(model, le, lr, status):
    lib = _lib.load()
    d, _buf = _desc(model, le, lr)
    out = (C.c_float * 4)()
    st = lib.kge_score(C.byref(d), 2, C.cast(out, C.c_void_p), C.cast(out, C.c_void_p), 1, 1,
                       C.cast(out, C.c_void_p), C.cast(out, C.c_void_p), None)
    assert st == status
    assert lib.kge_status_string(st)


def test_mode_validation():
    lib = _lib.load()
    d, _buf = _desc()
    p = C.cast((C.c_float * 4)(), C.c_void_p)
    assert lib.kge_score(C.byref(d), 9, p, p, 1, 1, p, p, None) == 2
    # train accepts only head-/tail-batch (dataloader.py:55-56)
    assert lib.kge_train_step_grads(C.byref(d), 0, p, p, 1, 1, p, None, 0, 0, 1, 1.0, 0.0, p, p, None, p, p,
                                    1 << 20, p, None) == 2


def test_workspace_checks():
    lib = _lib.load()
    d, _buf = _desc()
    p = C.cast((C.c_float * 4)(), C.c_void_p)
    need = lib.kge_train_workspace_bytes(C.byref(d), 4, 8)
    assert need > 0
    st = lib.kge_train_step_grads(C.byref(d), 2, p, p, 4, 8, p, None, 0, 0, 1, 1.0, 0.0, p, p, None, p, p,
                                  need - 1, p, None)
    assert st == 5
    assert lib.kge_rank_workspace_bytes(C.byref(d), 10) > 10 * 16 * 4


def test_python_errors_match_reference():
    from knowledgegraphembedding_amd import ops
    import torch
    with pytest.raises(ValueError, match="model Foo not supported"):
        ops.make_desc("Foo", torch.zeros(2, 2), torch.zeros(2, 2), 1.0, 1.0, None)
    with pytest.raises(RuntimeError, match="ROCm"):
        ops._require_device(torch.zeros(2))
