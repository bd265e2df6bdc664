"""The HIP entry points as PyTorch operators: torch.ops.kge.*.

SURVEY §8(b) names the drop-in boundary as a `kge` operator library
(`kge::score`, `kge::score_backward`, `kge::train_step_grads`,
`kge::rank_filtered`, `kge::sample_negatives`).  Each operator here is a
`torch.library.custom_op` whose implementation calls the extern "C" function
of libkge_hip.so (ops.py) on the current HIP stream; `register_fake` gives
the dispatcher the output metadata, so torch.compile / fake-tensor tracing
see one opaque node per call instead of a graph break, and `kge::score`
carries its autograd formula (`kge::score_backward`, the dense gradients the
reference's IndexSelectBackward + index_add_ produce).

Argument checks raise before any launch: ValueError with the reference's
messages for an unknown model or mode (model.py:64-70, 149, 162), RuntimeError
for tensors off the GPU (there is no CPU path), TypeError for dtypes.

    from knowledgegraphembedding_amd import torch_ops  # registers the ops
    s = torch.ops.kge.score(ent, rel, pos, neg, "tail-batch", "RotatE", 24.0, erange, None)
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from . import ops

_MODELS = ("TransE", "DistMult", "ComplEx", "RotatE", "pRotatE")
_MODES = ("single", "head-batch", "tail-batch")


def _check(model: str, mode: str, train: bool = False) -> None:
    if model not in _MODELS:
        raise ValueError("model %s not supported" % model)
    if mode not in _MODES or (train and mode == "single"):
        raise ValueError("mode %s not supported" % mode)


def _desc(model, entity, relation, gamma, erange, modulus):
    return ops.make_desc(model, entity.detach(), relation.detach(), gamma, erange,
                         None if modulus is None else modulus.detach())


# ------------------------------------------------------------------ score
@torch.library.custom_op("kge::score", mutates_args=())
def score(entity: Tensor, relation: Tensor, pos: Tensor, neg: Optional[Tensor], mode: str, model: str,
          gamma: float, embedding_range: float, modulus: Optional[Tensor]) -> Tensor:
    """KGEModel.forward (model.py:72-249): scores [B, n] ([B, 1] for 'single')."""
    _check(model, mode)
    dev = ops._require_device(entity, relation, pos, neg, modulus)
    return ops.score(_desc(model, entity, relation, gamma, embedding_range, modulus), mode, pos,
                     None if mode == "single" else neg, dev)


@score.register_fake
def _(entity, relation, pos, neg, mode, model, gamma, embedding_range, modulus):
    if mode == "single":
        return entity.new_empty(pos.shape[0], 1)
    return entity.new_empty(neg.shape[0], neg.shape[1])


@torch.library.custom_op("kge::score_backward", mutates_args=())
def score_backward(grad: Tensor, entity: Tensor, relation: Tensor, pos: Tensor, neg: Optional[Tensor], mode: str,
                   model: str, gamma: float, embedding_range: float,
                   modulus: Optional[Tensor]) -> tuple[Tensor, Tensor, Tensor]:
    """Dense d score / d (entity, relation, modulus) contracted with `grad`
    ([1, 1] modulus gradient for pRotatE, an empty tensor otherwise)."""
    _check(model, mode)
    dev = ops._require_device(grad, entity, relation, pos, neg, modulus)
    has_mod = modulus is not None
    ge, gr, gm = ops.score_backward(_desc(model, entity, relation, gamma, embedding_range, modulus), mode, pos,
                                    None if mode == "single" else neg, grad, dev, has_mod)
    return ge, gr, (gm.view(modulus.shape) if has_mod else entity.new_empty(0))


@score_backward.register_fake
def _(grad, entity, relation, pos, neg, mode, model, gamma, embedding_range, modulus):
    return (torch.empty_like(entity), torch.empty_like(relation),
            torch.empty_like(modulus) if modulus is not None else entity.new_empty(0))


def _score_setup(ctx, inputs, output):
    entity, relation, pos, neg, mode, model, gamma, erange, modulus = inputs
    ctx.save_for_backward(entity, relation, pos, neg, modulus)
    ctx.meta = (mode, model, gamma, erange)


def _score_bwd(ctx, grad):
    entity, relation, pos, neg, modulus = ctx.saved_tensors
    mode, model, gamma, erange = ctx.meta
    ge, gr, gm = torch.ops.kge.score_backward(grad.contiguous(), entity, relation, pos, neg, mode, model, gamma,
                                              erange, modulus)
    return ge, gr, None, None, None, None, None, None, (gm if modulus is not None else None)


torch.library.register_autograd("kge::score", _score_bwd, setup_context=_score_setup)


# ------------------------------------------------------------- train step
@torch.library.custom_op("kge::train_step_grads", mutates_args=())
def train_step_grads(entity: Tensor, relation: Tensor, modulus: Optional[Tensor], pos: Tensor, neg: Tensor,
                     subsampling_weight: Tensor, mode: str, model: str, gamma: float, embedding_range: float,
                     adversarial: bool, temperature: float, uni_weight: bool,
                     regularization: float) -> tuple[Tensor, Tensor, Tensor, Tensor]:
    """KGEModel.train_step up to loss.backward() (model.py:268-301), fused:
    (losses [4] = positive, negative, total loss, regularisation; dense
    entity gradient; dense relation gradient; modulus gradient [1, 1] for
    pRotatE, else empty)."""
    _check(model, mode, train=True)
    dev = ops._require_device(entity, relation, modulus, pos, neg, subsampling_weight)
    ge = torch.empty_like(entity, memory_format=torch.contiguous_format)
    gr = torch.empty_like(relation, memory_format=torch.contiguous_format)
    gm = torch.empty(1, 1, device=dev) if modulus is not None else entity.new_empty(0)
    losses = torch.empty(5, device=dev)
    ops.train_step_grads(_desc(model, entity, relation, gamma, embedding_range, modulus), mode, pos, neg,
                         subsampling_weight, dev, adversarial=adversarial, temperature=temperature,
                         uni_weight=uni_weight, regularization=regularization, grad_entity=ge, grad_relation=gr,
                         grad_modulus=gm if modulus is not None else None, losses=losses)
    return losses[:4].clone(), ge, gr, gm


@train_step_grads.register_fake
def _(entity, relation, modulus, pos, neg, subsampling_weight, mode, model, gamma, embedding_range, adversarial,
      temperature, uni_weight, regularization):
    return (entity.new_empty(4), torch.empty_like(entity), torch.empty_like(relation),
            entity.new_empty(1, 1) if modulus is not None else entity.new_empty(0))


# ------------------------------------------------------------------ ranking
@torch.library.custom_op("kge::rank_filtered", mutates_args=())
def rank_filtered(entity: Tensor, relation: Tensor, modulus: Optional[Tensor], queries: Tensor, filt_off: Tensor,
                  filt_ids: Tensor, mode: str, model: str, gamma: float, embedding_range: float,
                  path: str = "auto") -> tuple[Tensor, Tensor]:
    """Filtered ranks [nq] int64 and tie counts [nq] int32 of KGEModel.test_step
    (model.py:383-418, filter CSR from filters.FilterIndex)."""
    _check(model, mode, train=True)
    dev = ops._require_device(entity, relation, modulus, queries)
    return ops.rank_filtered(_desc(model, entity, relation, gamma, embedding_range, modulus), mode, queries,
                             filt_off, filt_ids, dev, path=path)


@rank_filtered.register_fake
def _(entity, relation, modulus, queries, filt_off, filt_ids, mode, model, gamma, embedding_range, path="auto"):
    nq = queries.shape[0]
    return queries.new_empty(nq, dtype=torch.int64), queries.new_empty(nq, dtype=torch.int32)


# ------------------------------------------------------------------ sampler
@torch.library.custom_op("kge::sample_negatives", mutates_args=("pos_out", "neg_out", "w_out"))
def sample_negatives(triples: Tensor, batch: Tensor, nentity: int, negative_sample_size: int, true_off: Tensor,
                     true_len: Tensor, true_ids: Tensor, weights: Tensor, key: int, max_draws: int, pos_out: Tensor,
                     neg_out: Tensor, w_out: Tensor) -> None:
    """TrainDataset.__getitem__ + collate_fn for one batch on the device
    (dataloader.py:34-66; kge_sample_negatives)."""
    ops.sample_negatives(triples, batch, nentity, negative_sample_size, true_off, true_len, true_ids, weights, key,
                         max_draws, pos_out, neg_out, w_out)


@sample_negatives.register_fake
def _(triples, batch, nentity, negative_sample_size, true_off, true_len, true_ids, weights, key, max_draws, pos_out,
      neg_out, w_out):
    return None
