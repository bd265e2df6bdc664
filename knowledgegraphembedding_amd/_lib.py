"""ctypes binding of the C-ABI in include/kge_hip.h.

The HIP library is the ONLY compute path of this package: if libkge_hip.so is
missing or a call fails, the error propagates — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("KGE_HIP_LIB", _PKG / "libkge_hip.so"))

# enum kge_model_id / kge_mode_id (include/kge_hip.h)
MODEL_IDS = {"TransE": 0, "DistMult": 1, "ComplEx": 2, "RotatE": 3, "pRotatE": 4}
MODE_IDS = {"single": 0, "head-batch": 1, "tail-batch": 2}
DEVERR_INDEX = 1
DEVERR_SAMPLER = 2
DEVERR_ARG = 4
ABI_VERSION = "0.5"  # KGE_ABI_VERSION of the include/kge_hip.h this binding mirrors
RANK_STAGE_LIST = 0x200  # KGE_RANK_STAGE_LIST
RANK_FILTER_TABLE = 0x400  # KGE_RANK_FILTER_TABLE
RANK_LIST_CAP = 1024  # KGE_RANK_LIST_CAP
PHASE_ROWS, PHASE_ENTITY, PHASE_FINALIZE, PHASE_ALL = 1, 2, 4, 7
SHIP_Q, SHIP_ROWS, SHIP_MERGE, SHIP_CHAIN, SHIP_ENTITY = 1, 2, 3, 4, 5
ERR_HIP_BASE = 1000


class ModelDesc(C.Structure):
    """struct kge_model_desc (struct_size is set on construction)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.struct_size = C.sizeof(ModelDesc)

    _fields_ = [
        ("model", C.c_int32),
        ("entity_dim", C.c_int32),
        ("relation_dim", C.c_int32),
        ("struct_size", C.c_int32),
        ("nentity", C.c_int64),
        ("nrelation", C.c_int64),
        ("gamma", C.c_float),
        ("phase_divisor", C.c_float),
        ("phase_divisor_p", C.c_float),
        ("reserved_f", C.c_float),
        ("entity_embedding", C.c_void_p),
        ("relation_embedding", C.c_void_p),
        ("modulus", C.c_void_p),
        ("relation_trig", C.c_void_p),
    ]


class AdamTensor(C.Structure):
    """struct kge_adam_tensor."""

    _fields_ = [("param", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("step_size", C.c_float), ("bias_correction2_sqrt", C.c_float)]


class AdamDesc(C.Structure):
    """struct kge_adam_desc."""

    _fields_ = [("entity", AdamTensor), ("relation", AdamTensor), ("modulus", AdamTensor),
                ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("write_grad", C.c_int32)]


class ShipDesc(C.Structure):
    """struct kge_ship_desc (query shipping, kge_ship_step)."""

    _fields_ = [("world", C.c_int32), ("rank", C.c_int32), ("own_begin", C.c_int64), ("own_end", C.c_int64),
                ("pos", C.c_void_p), ("neg", C.c_void_p), ("batch", C.c_int64), ("nneg", C.c_int64),
                ("subsampling_weight", C.c_void_p), ("weight_sum", C.c_void_p), ("uni_weight", C.c_int32),
                ("adversarial", C.c_int32), ("uni_batch", C.c_int64), ("adversarial_temperature", C.c_float),
                ("regularization", C.c_float), ("q", C.c_void_p), ("qp", C.c_void_p), ("part", C.c_void_p),
                ("parts", C.c_void_p), ("scores", C.c_void_p), ("g", C.c_void_p), ("dq", C.c_void_p),
                ("pq", C.c_void_p), ("pstats", C.c_void_p), ("ent_contrib", C.c_void_p),
                ("rel_contrib", C.c_void_p), ("row_stats", C.c_void_p)]


_P = C.c_void_p
_I32 = C.c_int32
_I64 = C.c_int64
_F = C.c_float
_SZ = C.c_size_t
_DESC = C.POINTER(ModelDesc)

# name -> (restype, argtypes); this table is also the symbol list the
# "library loads and exports every symbol" test checks against include/kge_hip.h.
SIGNATURES = {
    "kge_version": (C.c_char_p, []),
    "kge_status_string": (C.c_char_p, [C.c_int]),
    "kge_score": (C.c_int, [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _P]),
    "kge_backward_workspace_bytes": (_SZ, [_DESC, _I32, _I64, _I64]),
    "kge_score_backward": (C.c_int, [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _SZ, _P, _P]),
    "kge_train_workspace_bytes": (_SZ, [_DESC, _I64, _I64]),
    "kge_train_step_grads": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _I32, _F, _F, _P, _P, _P, _P, _P, _SZ, _P, _P],
    ),
    "kge_train_step_grads_phased": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _I32, _F, _F, _P, _P, _P, _P, _P, _SZ, _P, _P,
         _I32, _I64, _I64],
    ),
    "kge_train_step": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _I32, _F, _F, C.POINTER(AdamDesc), _P, _P, _P, _P, _P,
         _SZ, _P, _P],
    ),
    "kge_train_rows_slice": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _I32, _F, _P, _P, _P, _P, _SZ, _P, _P],
    ),
    "kge_train_step_from_rows": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _F, _P, _P, _P, C.POINTER(AdamDesc), _P, _P, _P, _P,
         _P, _SZ, _P, _P],
    ),
    "kge_train_csr": (C.c_int, [_DESC, _I32, _P, _P, _I64, _I64, _P, _SZ, _P, _P]),
    "kge_train_csr_range": (C.c_int, [_DESC, _I32, _P, _P, _I64, _I64, _I64, _I64, _P, _SZ, _P, _P]),
    "kge_train_step_from_rows_range": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _F, _P, _P, _P, C.POINTER(AdamDesc), _P, _P, _P, _P,
         _P, _SZ, _P, _P, _I64, _I64, _I32, _I32],
    ),
    "kge_train_step_from_rows_phased": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _F, _P, _P, _P, C.POINTER(AdamDesc), _P, _P, _P, _P,
         _P, _SZ, _P, _P, _I32, _I64, _I64, _I32, _I32],
    ),
    "kge_train_step_from_rows_csr": (
        C.c_int,
        [_DESC, _I32, _P, _P, _I64, _I64, _P, _P, _I32, _I64, _F, _P, _P, _P, C.POINTER(AdamDesc), _P, _P, _P, _P,
         _P, _SZ, _P, _P],
    ),
    "kge_ship_step": (C.c_int, [_DESC, _I32, C.POINTER(ShipDesc), _I32, C.POINTER(AdamDesc), _P, _P, _P, _P, _P,
                                _SZ, _P, _P]),
    "kge_weight_sum": (C.c_int, [_P, _I64, _P, _P]),
    "kge_adam_step": (C.c_int, [_P, _P, _P, _P, _I64, _F, _F, _F, _F, _F, _P]),
    "kge_rank_workspace_bytes": (_SZ, [_DESC, _I64]),
    "kge_rank_filtered": (C.c_int, [_DESC, _I32, _P, _I64, _P, _P, _P, _P, _P, _SZ, _P, _P]),
    "kge_rank_filtered_ex": (C.c_int, [_DESC, _I32, _P, _I64, _P, _P, _P, _P, _P, _I32, _P, _SZ, _P, _P]),
    "kge_rank_filtered_both": (C.c_int, [_DESC, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _SZ, _P, _P]),
    "kge_rank_sin_args": (C.c_int, [_DESC, _I32, _I64, _P, _P, _P, _SZ, _P, _P]),
    "kge_rank_finish_sin": (C.c_int, [_DESC, _I32, _I64, _P, _P, _P, _P, _P, _P, _SZ, _P, _P]),
    "kge_stage_timer": (C.c_int, [_I32, _P, _I32]),
    "kge_selftest_sin": (C.c_int, [C.c_float, _P, _P]),
    "kge_sample_negatives": (C.c_int, [_P, _I64, _P, _I64, _I64, _I64, _P, _P, _P, _P, C.c_uint64, _I64, _P, _P, _P,
                                       _P, _P]),
}

_lib = None


class KGEHipError(RuntimeError):
    pass


def load() -> C.CDLL:
    """Load libkge_hip.so (built by knowledgegraphembedding_amd.build) or raise."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise KGEHipError(
            f"{LIB_PATH} is missing: build it with `python -m knowledgegraphembedding_amd.build` "
            "(hipcc, gfx950). knowledgegraphembedding_amd has no CPU fallback."
        )
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    version = lib.kge_version().decode()
    if version.split()[1:2] != [ABI_VERSION]:
        raise KGEHipError(f"{LIB_PATH} reports ABI {version!r}; this binding mirrors kge_hip.h ABI {ABI_VERSION}: "
                          "rebuild the library (python -m knowledgegraphembedding_amd.build)")
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().kge_status_string(status).decode()
        if status == 1:
            raise ValueError(f"{what}: {msg}")
        raise KGEHipError(f"{what} failed with status {status}: {msg}")
