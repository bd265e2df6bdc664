"""The HIP entry points as PyTorch operators: torch.ops.kge.*.

SURVEY §8(b) names the drop-in boundary as a `kge` operator library.  It is
registered in C++ (`TORCH_LIBRARY(kge, m)`, csrc/torch/kge_torch_ops.cpp) and
built into libkge_torch.so next to the pure C-ABI libkge_hip.so; this module
only loads it (torch.ops.load_library), so a libtorch C++ caller links the
same library with no Python in the call path:

    kge::score(Tensor entity, Tensor relation, Tensor pos, Tensor? neg, int mode, int model,
               float gamma, float embedding_range, Tensor? modulus) -> Tensor
    kge::score_backward(Tensor grad, ...same...) -> (Tensor, Tensor, Tensor)
    kge::train_step_grads(Tensor entity, Tensor relation, Tensor? modulus, Tensor pos, Tensor neg,
                          Tensor subsampling_weight, int mode, int model, float gamma,
                          float embedding_range, bool adversarial, float temperature,
                          bool uni_weight, float regularization) -> (Tensor, Tensor, Tensor, Tensor)
    kge::rank_filtered(Tensor entity, Tensor relation, Tensor? modulus, Tensor queries,
                       Tensor filt_off, Tensor filt_ids, int mode, int model, float gamma,
                       float embedding_range, int path=0, Tensor? relation_trig=None)
                       -> (Tensor, Tensor)
    kge::sample_negatives(..., Tensor(a!) pos_out, Tensor(b!) neg_out, Tensor(c!) w_out) -> ()
    kge::error_flag(Device device) -> Tensor

`model` / `mode` are the integer ids of include/kge_hip.h (MODEL_IDS /
MODE_IDS below).  The C++ side registers CUDA kernels (the C-ABI on the
current HIP stream), Meta kernels (output metadata, so torch.compile /
fake-tensor tracing carry one opaque node per call), CPU kernels that refuse
(there is no CPU path) and kge::score's autograd (kge::score_backward, the
dense gradients the reference's IndexSelectBackward + index_add_ produce).
Argument checks are TORCH_CHECKs raised before any launch: ValueError with
the reference's messages for an unknown model or mode (model.py:64-70, 149,
162), RuntimeError for devices, dtypes and shapes.

    from knowledgegraphembedding_amd import torch_ops  # loads libkge_torch.so
    s = torch.ops.kge.score(ent, rel, pos, neg, torch_ops.MODE_IDS["tail-batch"],
                            torch_ops.MODEL_IDS["RotatE"], 24.0, erange, None)
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

from ._lib import MODE_IDS, MODEL_IDS  # noqa: F401  (re-exported: the ops' integer ids)

LIB_PATH = Path(os.environ.get("KGE_TORCH_LIB", Path(__file__).resolve().parent / "libkge_torch.so"))
_LOADED = [False]


def load() -> None:
    """Register torch.ops.kge.* from libkge_torch.so (once), or raise: every
    entry point of the package calls this before its first torch.ops.kge op."""
    if _LOADED[0]:
        return
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m knowledgegraphembedding_amd.build` "
                           "(the kge operator library; knowledgegraphembedding_amd has no CPU fallback)")
    torch.ops.load_library(str(LIB_PATH))
    _LOADED[0] = True


# registered at import when built; a fresh checkout can still be imported to
# build it (`build.py` imports the package), and its first op raises above
if LIB_PATH.exists():
    load()
