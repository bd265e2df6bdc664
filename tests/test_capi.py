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
    # (any row length is accepted since round 5: (half-)rows over 2048 floats
    # run kge_wide.inc's kernels, tests/test_wide_gpu.py — a valid shape would
    # launch, so none is checked here)
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


def test_abi_version_and_struct_size():
    """a caller built against another kge_model_desc layout is
    refused (KGE_ERR_ABI) instead of reading past its struct; the loader
    refuses a library of another ABI version."""
    lib = _lib.load()
    assert lib.kge_version().decode().split()[1] == _lib.ABI_VERSION
    d, _buf = _desc()
    assert d.struct_size == C.sizeof(_lib.ModelDesc)
    out = (C.c_float * 4)()
    p = C.cast(out, C.c_void_p)
    d.struct_size = C.sizeof(_lib.ModelDesc) - 8  # an older, shorter struct
    st = lib.kge_score(C.byref(d), 2, p, p, 1, 1, p, p, None)
    assert st == 7 and b"struct_size" in lib.kge_status_string(st)
    d.struct_size = 0  # the round-3 layout's "reserved" word
    assert lib.kge_rank_workspace_bytes(C.byref(d), 4) > 0  # (sizes only; no validation there)
    assert lib.kge_rank_filtered(C.byref(d), 2, p, 1, p, p, p, p, p, 1 << 20, p, None) == 7


def test_protate_library_sin_stage_checks():
    """The three-call pRotatE form accepts only pRotatE and needs its buffers
    (checked on the host before any launch)."""
    lib = _lib.load()
    p = C.cast((C.c_float * 4)(), C.c_void_p)
    d, _buf = _desc(3, 16, 8)  # RotatE
    assert lib.kge_rank_sin_args(C.byref(d), 2, 1, p, p, p, 1 << 20, p, None) == 1
    assert lib.kge_rank_finish_sin(C.byref(d), 2, 1, p, p, p, p, None, p, 1 << 20, p, None) == 1
    d, _buf = _desc(4, 16, 16)  # pRotatE
    assert lib.kge_rank_sin_args(C.byref(d), 2, 1, None, p, p, 1 << 20, p, None) == 4
    assert lib.kge_rank_finish_sin(C.byref(d), 2, 1, p, None, p, p, None, p, 1 << 20, p, None) == 4
    assert lib.kge_rank_filtered_ex(C.byref(d), 2, p, 1, p, p, p, p, None, _lib.RANK_STAGE_LIST, p, 1 << 20, p,
                                    None) == 4  # the list stage must return the counts
    assert lib.kge_rank_sin_args(C.byref(d), 2, 1, p, p, p, 16, p, None) == 5  # workspace
