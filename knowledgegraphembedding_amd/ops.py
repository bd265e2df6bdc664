"""Torch-facing wrappers of the HIP entry points (include/kge_hip.h).

PyTorch supplies device memory and the current HIP stream; every FLOP of the
hot path runs in libkge_hip.so.  Tensors must live on a ROCm device: there is
deliberately no CPU path (a CPU fallback would void the parity claims).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch

from . import _lib

PI = 3.14159265358979323846   # model.py:202
PI_TYPO = 3.14159262358979323846  # model.py:232 (pRotatE; reproduced on purpose)


def _require_device(*ts: torch.Tensor) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "knowledgegraphembedding_amd runs on MI355X (ROCm) only: got a tensor on "
                f"{t.device}. Move the model and batch to the GPU (run.py --cuda)."
            )
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} vs {t.device}")
    return dev


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


class _DeviceState:
    """Per-device scratch: a growable workspace per HIP stream, and the device
    error flag (written only by atomic OR, so streams may share it).

    Calls enqueued on one stream use that stream's workspace, so work issued
    from two torch streams at once never shares scratch memory; a workspace
    is replaced (not resized in place) when a larger call comes, and the
    caching allocator keeps the old block until the stream has moved past it."""

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.ws = {}
        self.rank_ws_ptr = 0  # workspace of the last ranking call (KGE_RANK_REUSE_TABLE)
        # the flag the torch.ops.kge.* kernels OR into too (one per device)
        from . import torch_ops
        torch_ops.load()
        self.err = torch.ops.kge.error_flag(dev)

    def workspace(self, nbytes: int) -> torch.Tensor:
        self.rank_ws_ptr = 0  # any user may overwrite the ranking's reusable table buffers
        s = torch.cuda.current_stream(self.dev)
        key = s.cuda_stream
        ws = self.ws.get(key)
        if ws is None or ws.numel() < nbytes:
            ws = self.ws[key] = torch.empty(int(nbytes * 1.25) + 4096, dtype=torch.uint8, device=self.dev)
        return ws


_STATES: dict = {}
_WS_BYTES: dict = {}  # (dims, counts, B, n) -> kge_train_workspace_bytes


def state(dev: torch.device) -> _DeviceState:
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    st = _STATES.get(key)
    if st is None:
        st = _STATES[key] = _DeviceState(torch.device("cuda", key[1]))
    return st


def raise_on_device_error(dev: torch.device) -> None:
    """Read (and clear) the device error flag — a sync point."""
    raise_device_error_value(dev, int(state(dev).err.item()))


def raise_device_error_value(dev: torch.device, v: int) -> None:
    """Raise for an error-flag value already read back (and clear the flag)."""
    st = state(dev)
    if v:
        st.err.zero_()
        if v & _lib.DEVERR_INDEX:
            raise IndexError("index out of range in self")  # what index_select raises (model.py:86-146)
        if v & _lib.DEVERR_SAMPLER:
            raise RuntimeError("negative sampler: a positive's true heads/tails leave too few candidate "
                               "entities (the reference's sampling loop would not terminate)")
        if v & _lib.DEVERR_ARG:
            raise RuntimeError("pRotatE three-call ranking: item offsets do not match the listed near-tie counts, or the "
                               "call does not follow its list stage (mode, nq, table or workspace changed)")
        raise RuntimeError(f"device error flag {v}")


def phase_divisors(embedding_range: float) -> tuple[float, float]:
    """(range/pi, range/pi') in double, as model.py:209 / :236 compute them."""
    return embedding_range / PI, embedding_range / PI_TYPO


def make_desc(model_name: str, entity: torch.Tensor, relation: torch.Tensor, gamma: float, embedding_range: float,
              modulus: Optional[torch.Tensor]) -> _lib.ModelDesc:
    if model_name not in _lib.MODEL_IDS:
        raise ValueError("model %s not supported" % model_name)
    if entity.dtype != torch.float32 or relation.dtype != torch.float32:
        raise TypeError("embeddings must be float32 (model.py:45,52)")
    if not (entity.is_contiguous() and relation.is_contiguous()):
        raise ValueError("embeddings must be contiguous")
    k, kp = phase_divisors(embedding_range)
    d = _lib.ModelDesc()
    d.model = _lib.MODEL_IDS[model_name]
    d.entity_dim = entity.shape[1]
    d.relation_dim = relation.shape[1]
    d.nentity = entity.shape[0]
    d.nrelation = relation.shape[0]
    d.gamma = gamma
    d.phase_divisor = k
    d.phase_divisor_p = kp
    d.entity_embedding = entity.data_ptr()
    d.relation_embedding = relation.data_ptr()
    d.modulus = modulus.data_ptr() if modulus is not None else None
    return d


def _idx(t: torch.Tensor, dev) -> torch.Tensor:
    if t.device != dev:
        t = t.to(dev, non_blocking=True)
    if t.dtype != torch.int64:
        t = t.long()
    return t.contiguous()


def score(desc: _lib.ModelDesc, mode: str, pos: torch.Tensor, neg: Optional[torch.Tensor], dev) -> torch.Tensor:
    """Scores [B, n] (model.py:72-249)."""
    if mode not in _lib.MODE_IDS:
        raise ValueError("mode %s not supported" % mode)
    pos = _idx(pos, dev)
    if mode == "single":
        B, n = pos.shape[0], 1
        neg = None
    else:
        neg = _idx(neg, dev)
        B, n = neg.shape[0], neg.shape[1]
    out = torch.empty(B, n, dtype=torch.float32, device=dev)
    st = state(dev)
    lib = _lib.load()
    _lib.check(
        lib.kge_score(desc, _lib.MODE_IDS[mode], pos.data_ptr(), _ptr(neg), B, n, out.data_ptr(),
                      st.err.data_ptr(), _stream(dev)),
        "kge_score",
    )
    return out


def score_backward(desc: _lib.ModelDesc, mode: str, pos: torch.Tensor, neg: Optional[torch.Tensor],
                   grad_scores: torch.Tensor, dev, with_modulus: bool):
    pos = _idx(pos, dev)
    if mode == "single":
        neg = None
        B, n = pos.shape[0], 1
    else:
        neg = _idx(neg, dev)
        B, n = neg.shape
    g = grad_scores.to(torch.float32).contiguous().view(B, n)
    ge = torch.empty(desc.nentity, desc.entity_dim, dtype=torch.float32, device=dev)
    gr = torch.empty(desc.nrelation, desc.relation_dim, dtype=torch.float32, device=dev)
    gm = torch.empty(1, 1, dtype=torch.float32, device=dev) if with_modulus else None
    lib = _lib.load()
    m = _lib.MODE_IDS[mode]
    need = lib.kge_backward_workspace_bytes(desc, m, B, n)
    st = state(dev)
    ws = st.workspace(need)
    _lib.check(
        lib.kge_score_backward(desc, m, pos.data_ptr(), _ptr(neg), B, n, g.data_ptr(), ge.data_ptr(), gr.data_ptr(),
                               _ptr(gm), ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev)),
        "kge_score_backward",
    )
    return ge, gr, gm


def weight_sum(w: torch.Tensor, out: torch.Tensor) -> None:
    dev = w.device
    _lib.check(_lib.load().kge_weight_sum(w.data_ptr(), w.numel(), out.data_ptr(), _stream(dev)), "kge_weight_sum")


def train_step_grads(desc: _lib.ModelDesc, mode: str, pos: torch.Tensor, neg: torch.Tensor, sub_w: torch.Tensor,
                     dev, *, adversarial: bool, temperature: float, uni_weight: bool, regularization: float,
                     grad_entity: torch.Tensor, grad_relation: torch.Tensor, grad_modulus: Optional[torch.Tensor],
                     losses: torch.Tensor, weight_sum_dev: Optional[torch.Tensor] = None,
                     uni_batch: int = 0, adam: Optional[_lib.AdamDesc] = None, phases: int = _lib.PHASE_ALL,
                     entity_range: Optional[tuple] = None) -> None:
    """Fused scoring + loss + backward into the given dense grad buffers (model.py:252-301);
    with `adam`, also the optimizer step, fused into the gradient passes (model.py:303).
    `phases` / `entity_range` run a part of the step (kge_train_step_grads_phased): the
    data-parallel path reduces entity-row chunks while later chunks are computed."""
    if mode not in ("head-batch", "tail-batch"):
        raise ValueError("Training batch mode %s not supported" % mode)
    pos = _idx(pos, dev)
    neg = _idx(neg, dev)
    w = sub_w.to(dev, dtype=torch.float32, non_blocking=True).contiguous().view(-1)
    B, n = neg.shape
    lib = _lib.load()
    key = (desc.entity_dim, desc.relation_dim, desc.nentity, desc.nrelation, B, n)
    need = _WS_BYTES.get(key)
    if need is None:
        need = _WS_BYTES[key] = lib.kge_train_workspace_bytes(desc, B, n)
    st = state(dev)
    ws = st.workspace(need)
    common = (desc, _lib.MODE_IDS[mode], pos.data_ptr(), neg.data_ptr(), B, n, w.data_ptr(), _ptr(weight_sum_dev),
              int(bool(uni_weight)), int(uni_batch), int(bool(adversarial)), float(temperature), float(regularization))
    tail = (grad_entity.data_ptr(), grad_relation.data_ptr(), _ptr(grad_modulus), losses.data_ptr(), ws.data_ptr(),
            ws.numel(), st.err.data_ptr(), _stream(dev))
    if phases != _lib.PHASE_ALL or entity_range is not None:
        if adam is not None:
            raise ValueError("phased train steps take no fused optimizer")
        e0, e1 = entity_range if entity_range is not None else (0, desc.nentity)
        _lib.check(lib.kge_train_step_grads_phased(*common, *tail, int(phases), int(e0), int(e1)),
                   "kge_train_step_grads_phased")
    elif adam is None:
        _lib.check(lib.kge_train_step_grads(*common, *tail), "kge_train_step_grads")
    else:
        _lib.check(lib.kge_train_step(*common, adam, *tail), "kge_train_step")


def _train_ws(desc: _lib.ModelDesc, B: int, n: int, dev) -> torch.Tensor:
    lib = _lib.load()
    key = (desc.entity_dim, desc.relation_dim, desc.nentity, desc.nrelation, B, n)
    need = _WS_BYTES.get(key)
    if need is None:
        need = _WS_BYTES[key] = lib.kge_train_workspace_bytes(desc, B, n)
    return state(dev).workspace(need)


_AUX_WS: dict = {}


def exchange_workspace(desc: _lib.ModelDesc, B: int, n: int, dev) -> torch.Tensor:
    """A step workspace of its own for the factor exchange's global batch:
    train_csr runs on a side stream while this rank's row pass (which uses the
    shared per-device workspace) is still running, so the two must not share
    memory.  Grown (after a device sync) only when a larger batch comes."""
    lib = _lib.load()
    key = (desc.entity_dim, desc.relation_dim, desc.nentity, desc.nrelation, B, n)
    need = _WS_BYTES.get(key)
    if need is None:
        need = _WS_BYTES[key] = lib.kge_train_workspace_bytes(desc, B, n)
    t = _AUX_WS.get(dev)
    if t is None or t.numel() < need:
        if t is not None:
            torch.cuda.synchronize(dev)  # the old buffer may still be read on either stream
        t = _AUX_WS[dev] = torch.empty(int(need * 1.25) + 4096, dtype=torch.uint8, device=dev)
    return t


def _check_row_buffers(dev, B: int, n: int, Le: int, g, dq, stats) -> None:
    for t, shape in ((g, (B, n)), (dq, (B, Le)), (stats, (B, 4))):
        if (tuple(t.shape) != shape or not t.is_contiguous() or t.dtype != torch.float32
                or t.device != dev):
            raise ValueError(f"row buffer {tuple(t.shape)} {t.dtype} on {t.device}: expected contiguous "
                             f"float32 {shape} on {dev}")


def train_rows_slice(desc: _lib.ModelDesc, mode: str, pos: torch.Tensor, neg: torch.Tensor, sub_w: torch.Tensor,
                     weight_sum_dev: Optional[torch.Tensor], dev, *, adversarial: bool, temperature: float,
                     uni_weight: bool, uni_batch: int, g_out: torch.Tensor, dq_out: torch.Tensor,
                     stats_out: torch.Tensor) -> None:
    """The negative-row pass alone for this rank's rows (kge_train_rows_slice):
    dL/ds, dL/dq and the row statistics into the rank's place in the gather
    buffers (the data-parallel factor exchange, distributed.py)."""
    if mode not in ("head-batch", "tail-batch"):
        raise ValueError("Training batch mode %s not supported" % mode)
    pos, neg = _idx(pos, dev), _idx(neg, dev)
    w = sub_w.to(dev, dtype=torch.float32).contiguous().view(-1)
    B, n = neg.shape
    _check_row_buffers(dev, B, n, desc.entity_dim, g_out, dq_out, stats_out)
    ws = _train_ws(desc, B, n, dev)
    st = state(dev)
    _lib.check(_lib.load().kge_train_rows_slice(
        desc, _lib.MODE_IDS[mode], pos.data_ptr(), neg.data_ptr(), B, n, w.data_ptr(), _ptr(weight_sum_dev),
        int(bool(uni_weight)), int(uni_batch), int(bool(adversarial)), float(temperature), g_out.data_ptr(),
        dq_out.data_ptr(), stats_out.data_ptr(), ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev)),
        "kge_train_rows_slice")


def train_csr(desc: _lib.ModelDesc, mode: str, pos: torch.Tensor, neg: torch.Tensor, dev,
              workspace: Optional[torch.Tensor] = None, entity_range: Optional[tuple] = None) -> None:
    """The occurrence CSR of the (gathered) batch into a step workspace
    (kge_train_csr), ahead of train_step_from_rows(..., csr_ready=True) with
    the SAME workspace — it needs only the ids, so it runs while the row
    factors are on the wire.  With `entity_range` (e0, e1) only those
    entities' buckets are built (kge_train_csr_range: an owner's rows)."""
    if mode not in ("head-batch", "tail-batch"):
        raise ValueError("Training batch mode %s not supported" % mode)
    pos, neg = _idx(pos, dev), _idx(neg, dev)
    B, n = neg.shape
    ws = workspace if workspace is not None else _train_ws(desc, B, n, dev)
    st = state(dev)
    lib = _lib.load()
    if entity_range is not None:
        e0, e1 = entity_range
        _lib.check(lib.kge_train_csr_range(desc, _lib.MODE_IDS[mode], pos.data_ptr(), neg.data_ptr(), B, n, int(e0),
                                           int(e1), ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev)),
                   "kge_train_csr_range")
        return
    _lib.check(lib.kge_train_csr(desc, _lib.MODE_IDS[mode], pos.data_ptr(), neg.data_ptr(), B, n,
                                 ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev)), "kge_train_csr")


def train_step_from_rows(desc: _lib.ModelDesc, mode: str, pos: torch.Tensor, neg: torch.Tensor, sub_w: torch.Tensor,
                         weight_sum_dev: Optional[torch.Tensor], dev, *, uni_weight: bool, uni_batch: int,
                         regularization: float, g_in: torch.Tensor, dq_in: torch.Tensor, stats: torch.Tensor,
                         grad_entity: torch.Tensor, grad_relation: torch.Tensor, grad_modulus: Optional[torch.Tensor],
                         losses: torch.Tensor, adam: Optional[_lib.AdamDesc] = None, csr_ready: bool = False,
                         workspace: Optional[torch.Tensor] = None, entity_range: Optional[tuple] = None,
                         reg_relations: bool = True, phases: Optional[int] = None) -> None:
    """The rest of the step for the whole (gathered) batch from the exchanged
    row factors (kge_train_step_from_rows; with csr_ready the CSR train_csr
    built for this batch, kge_train_step_from_rows_csr); bit-identical to one
    process running train_step_grads / the fused step on that batch.  With
    `entity_range` (e0, e1) the entity-major pass and its Adam cover only those
    rows (the owner-computes step, kge_train_step_from_rows_range); with
    `phases` as well, only those phases run (PHASE_ROWS / PHASE_ENTITY /
    PHASE_FINALIZE, kge_train_step_from_rows_phased)."""
    if mode not in ("head-batch", "tail-batch"):
        raise ValueError("Training batch mode %s not supported" % mode)
    pos, neg = _idx(pos, dev), _idx(neg, dev)
    w = sub_w.to(dev, dtype=torch.float32).contiguous().view(-1)
    B, n = neg.shape
    _check_row_buffers(dev, B, n, desc.entity_dim, g_in, dq_in, stats)
    ws = workspace if workspace is not None else _train_ws(desc, B, n, dev)
    st = state(dev)
    args = (desc, _lib.MODE_IDS[mode], pos.data_ptr(), neg.data_ptr(), B, n, w.data_ptr(), _ptr(weight_sum_dev),
            int(bool(uni_weight)), int(uni_batch), float(regularization), g_in.data_ptr(), dq_in.data_ptr(),
            stats.data_ptr(), adam, grad_entity.data_ptr(), grad_relation.data_ptr(), _ptr(grad_modulus),
            losses.data_ptr(), ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev))
    if phases is not None:
        e0, e1 = entity_range if entity_range is not None else (0, desc.nentity)
        _lib.check(_lib.load().kge_train_step_from_rows_phased(*args, int(phases), int(e0), int(e1),
                                                               int(bool(csr_ready)), int(bool(reg_relations))),
                   "kge_train_step_from_rows_phased")
        return
    if entity_range is not None:
        e0, e1 = entity_range
        _lib.check(_lib.load().kge_train_step_from_rows_range(*args, int(e0), int(e1), int(bool(csr_ready)),
                                                              int(bool(reg_relations))),
                   "kge_train_step_from_rows_range")
        return
    fn = "kge_train_step_from_rows_csr" if csr_ready else "kge_train_step_from_rows"
    _lib.check(getattr(_lib.load(), fn)(*args), fn)


def ship_step(desc: _lib.ModelDesc, mode: str, stage: int, ship: _lib.ShipDesc, dev, *,
              adam: Optional[_lib.AdamDesc] = None, grad_entity_ptr: int = 0,
              grad_relation: Optional[torch.Tensor] = None, grad_modulus: Optional[torch.Tensor] = None,
              losses: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None) -> None:
    """One stage of the query-shipping step (kge_ship_step; partition.py
    exchange "queries" drives the stages and the collectives between them).
    `desc` and `grad_entity_ptr` address the shard by GLOBAL row id (base
    pointers own_begin rows before the shard)."""
    if mode not in ("head-batch", "tail-batch"):
        raise ValueError("Training batch mode %s not supported" % mode)
    ws = workspace if workspace is not None else _train_ws(desc, ship.batch, ship.nneg, dev)
    st = state(dev)
    _lib.check(_lib.load().kge_ship_step(desc, _lib.MODE_IDS[mode], ship, int(stage), adam, grad_entity_ptr or None,
                                         _ptr(grad_relation), _ptr(grad_modulus), _ptr(losses), ws.data_ptr(),
                                         ws.numel(), st.err.data_ptr(), _stream(dev)), "kge_ship_step")


def adam_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, *,
              step: int, lr: float, beta1: float, beta2: float, eps: float) -> None:
    """torch.optim.Adam's update for one tensor (bias corrections in double, like torch)."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    bc2_sqrt = math.sqrt(bc2)
    dev = _require_device(param, grad, exp_avg, exp_avg_sq)
    for t in (param, grad, exp_avg, exp_avg_sq):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise ValueError("adam tensors must be contiguous float32")
    _lib.check(
        _lib.load().kge_adam_step(param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                                  param.numel(), beta1, beta2, eps, step_size, bc2_sqrt, _stream(dev)),
        "kge_adam_step",
    )


RANK_PATHS = {"auto": 0, "mfma": 1, "tile": 2, "scan": 3, "mfma32": 4}


def reference_rotation(relation: torch.Tensor, embedding_range: float) -> torch.Tensor:
    """RotatE's relation rotations as the reference evaluates them: [R, 2, d]
    (cos θ | sin θ) of θ = relation / (embedding_range / π), by the
    reference's own ATen CPU ops (model.py:209-212) — the table
    kge_model_desc.relation_trig carries into the filtered ranking.

    Only this [R, d] table is evaluated on the host, once per ranking call:
    the reference's ranks are defined by its CPU vector library's cos / sin,
    which no device instruction sequence reproduces bit for bit (they differ
    from correctly rounded values on ~5 % of arguments).  Elementwise, so the
    whole table gives the same bits as the reference's gathered [B, 1, d]
    rows (tests/test_rank_parity_gpu.py checks the host's bits against the
    reference's, committed in tests/golden/rotate_trig.npz)."""
    rel = relation.detach().to("cpu", torch.float32)
    phase = rel / (embedding_range / PI)
    return torch.stack([torch.cos(phase), torch.sin(phase)], 1).contiguous()


RANK_REUSE_TABLE = 0x100  # kge_hip.h KGE_RANK_REUSE_TABLE


def _check_filter_shape(desc, nq: int, off: torch.Tensor, filter_table: bool) -> None:
    """The device reads filt_off at every query's key (whole index, E·R + 1
    starts) or at q, q + 1 (per-query lists, nq + 1): a wrong-sized array is
    an out-of-bounds read on the device, refused here."""
    want = desc.nentity * desc.nrelation + 1 if filter_table else nq + 1
    if off.dim() != 1 or off.numel() != want:
        raise ValueError(f"filter offsets: {tuple(off.shape)}, expected [{want}] "
                         f"({'the whole index, E·R + 1' if filter_table else 'per-query lists, nq + 1'})")


def rank_filtered(desc: _lib.ModelDesc, mode: str, queries: torch.Tensor, filt_off: torch.Tensor,
                  filt_ids: torch.Tensor, dev, path: str = "auto", listed: bool = False,
                  relation_trig: Optional[torch.Tensor] = None, reuse_table: bool = False,
                  library_sin: bool = False, filter_table: bool = False):
    """Filtered ranks (int64) and tie counts (int32) for a block of queries
    (model.py:383-418), in the reference's fp32 score order
    (kge_rank_filtered_ex).  `path` picks the fast counting pass ("auto",
    "mfma" = split-bf16 MFMA tile, "mfma32" = fp32 MFMA tile, "tile", "scan"); `listed` also returns the per-query number of
    near-ties that were re-scored; `relation_trig` (RotatE, [R, 2, d] on the
    device, see reference_rotation) is the rotation table the ranks are
    computed with (None: correctly rounded cos / sin).  `reuse_table`: an
    earlier call on this device ranked the same model with the same, unchanged
    entity table (the other direction or another query block of one
    evaluation) — its table statistics and split operands are reused when the
    shared workspace is still the same buffer (else recomputed).
    `library_sin` (pRotatE): evaluate the sin of the near-ties' phase sums
    with the reference's own torch.sin on the host (reference_sin), so the
    ranks are the reference's bit for bit; False: correctly rounded device sin.
    `filter_table`: filt_off / filt_ids are the whole filter index
    (FilterIndex.device_table: dense key → start table and the sorted ids)
    instead of per-query lists; the device looks each query's list up."""
    if mode not in ("head-batch", "tail-batch"):
        raise ValueError("mode %s not supported" % mode)
    if path not in RANK_PATHS:
        raise ValueError("rank path %s not supported" % path)
    if relation_trig is not None:
        shape = (desc.nrelation, 2, desc.relation_dim)
        if (tuple(relation_trig.shape) != shape or relation_trig.dtype != torch.float32
                or not relation_trig.is_contiguous() or relation_trig.device != dev):
            raise ValueError(f"relation_trig: expected a contiguous float32 {shape} tensor on {dev}")
        desc = _lib.ModelDesc.from_buffer_copy(desc)
        desc.relation_trig = relation_trig.data_ptr()
    q = _idx(queries, dev)
    _check_filter_shape(desc, q.shape[0], filt_off, filter_table)
    off = _idx(filt_off, dev)
    ids = _idx(filt_ids, dev) if filt_ids.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
    nq = q.shape[0]
    ranks = torch.empty(nq, dtype=torch.int64, device=dev)
    ties = torch.empty(nq, dtype=torch.int32, device=dev)
    lst = torch.empty(nq, dtype=torch.int32, device=dev) if listed else None
    lib = _lib.load()
    need = lib.kge_rank_workspace_bytes(desc, nq)
    st = state(dev)
    key = (desc.entity_embedding, desc.nentity, desc.entity_dim, desc.model)
    prev = st.rank_ws_ptr  # the last ranking call's (buffer, table), cleared by any other workspace user
    ws = st.workspace(need)
    # the table's statistics / split operands survive only in the same buffer
    # (the library also checks its own tag of what the buffer holds)
    reuse_table = reuse_table and prev == (ws.data_ptr(),) + key
    st.rank_ws_ptr = (ws.data_ptr(),) + key
    flags = RANK_PATHS[path] | (RANK_REUSE_TABLE if reuse_table else 0) | (_lib.RANK_FILTER_TABLE if filter_table else 0)
    mode_id = _lib.MODE_IDS[mode]
    if library_sin and desc.model == _lib.MODEL_IDS["pRotatE"] and nq:
        _rank_protate_library_sin(lib, desc, mode_id, q, nq, off, ids, ranks, ties, lst, flags, ws, st, dev)
    else:
        _lib.check(
            lib.kge_rank_filtered_ex(desc, mode_id, q.data_ptr(), nq, off.data_ptr(), ids.data_ptr(),
                                     ranks.data_ptr(), ties.data_ptr(), _ptr(lst), flags, ws.data_ptr(),
                                     ws.numel(), st.err.data_ptr(), _stream(dev)),
            "kge_rank_filtered_ex",
        )
    return (ranks, ties, lst) if listed else (ranks, ties)


def rank_filtered_both(desc: _lib.ModelDesc, queries: torch.Tensor, filt_head, filt_tail, dev, path: str = "auto",
                       listed: bool = False, relation_trig: Optional[torch.Tensor] = None, reuse_table: bool = False,
                       filter_table: bool = False, out: Optional[torch.Tensor] = None):
    """Both directions of one evaluation in one pass (kge_rank_filtered_both):
    ranks [2·nq] int64 and ties [2·nq] int32 — head-batch then tail-batch, the
    same values as rank_filtered(mode="head-batch") then
    rank_filtered(mode="tail-batch").  filt_head / filt_tail: each direction's
    (filt_off, filt_ids), per-query lists or (filter_table) the whole index.
    `queries` may be a (pinned) host tensor: it is copied right before the
    launch, after the host-side preparation, so the device does not wait for
    Python between the copy and the first kernel.  `out` (int32 [6·nq] on the
    device): ranks and ties written into it as [ranks as int32 pairs | ties],
    one buffer for the caller's single read-back.  Not for pRotatE with the
    reference's library sin (per direction: rank_filtered's three-call form)."""
    if path not in RANK_PATHS:
        raise ValueError("rank path %s not supported" % path)
    if relation_trig is not None:
        shape = (desc.nrelation, 2, desc.relation_dim)
        if (tuple(relation_trig.shape) != shape or relation_trig.dtype != torch.float32
                or not relation_trig.is_contiguous() or relation_trig.device != dev):
            raise ValueError(f"relation_trig: expected a contiguous float32 {shape} tensor on {dev}")
        desc = _lib.ModelDesc.from_buffer_copy(desc)
        desc.relation_trig = relation_trig.data_ptr()
    nq = queries.shape[0]
    _check_filter_shape(desc, nq, filt_head[0], filter_table)
    _check_filter_shape(desc, nq, filt_tail[0], filter_table)
    fl = []
    for off, ids in (filt_head, filt_tail):
        fl.append((_idx(off, dev), _idx(ids, dev) if ids.numel() else torch.zeros(1, dtype=torch.int64, device=dev)))
    if out is None:
        ranks = torch.empty(2 * nq, dtype=torch.int64, device=dev)
        ties = torch.empty(2 * nq, dtype=torch.int32, device=dev)
    else:
        if out.dtype != torch.int32 or out.device != dev or out.numel() < 6 * nq or not out.is_contiguous():
            raise ValueError("out: a contiguous int32 device tensor of at least 6·nq elements")
        ranks, ties = out[:4 * nq].view(torch.int64), out[4 * nq:6 * nq]
    lst = torch.empty(2 * nq, dtype=torch.int32, device=dev) if listed else None
    lib = _lib.load()
    need = lib.kge_rank_workspace_bytes(desc, 2 * nq)
    st = state(dev)
    key = (desc.entity_embedding, desc.nentity, desc.entity_dim, desc.model)
    prev = st.rank_ws_ptr
    ws = st.workspace(need)
    reuse_table = reuse_table and prev == (ws.data_ptr(),) + key
    st.rank_ws_ptr = (ws.data_ptr(),) + key
    flags = RANK_PATHS[path] | (RANK_REUSE_TABLE if reuse_table else 0) | (_lib.RANK_FILTER_TABLE if filter_table else 0)
    q = _idx(queries, dev)  # (a pinned host tensor: its copy queues right before the launch)
    _lib.check(lib.kge_rank_filtered_both(desc, q.data_ptr(), nq, fl[0][0].data_ptr(), fl[0][1].data_ptr(),
                                          fl[1][0].data_ptr(), fl[1][1].data_ptr(), ranks.data_ptr(), ties.data_ptr(),
                                          _ptr(lst), flags, ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev)),
               "kge_rank_filtered_both")
    return (ranks, ties, lst) if listed else (ranks, ties)


def reference_sin(args: torch.Tensor) -> torch.Tensor:
    """sin of pRotatE phase sums as the reference evaluates them: its own
    `torch.sin` on the CPU (model.py:245; ATen's vectorized CPU kernel — MKL
    VML in this build — whose last bits no device instruction sequence
    reproduces).  Elementwise, so the values do not depend on how the
    arguments are batched (tests/test_rank_parity_gpu.py checks this host's
    bits against the reference's, tests/golden/protate_sin.npz)."""
    return torch.sin(args)


def device_sin_queries(dev, reset: bool = True) -> int:
    """pRotatE with the library sin: how many queries since the last reset the
    list stage ranked with correctly rounded device sin instead (more
    undecided candidates than RANK_LIST_CAP; each such call also logs a
    warning).  0 means every pRotatE rank so far is the reference's bit for bit."""
    st = state(dev)
    n = st.__dict__.get("device_sin_queries", 0)
    if reset:
        st.__dict__["device_sin_queries"] = 0
    return n


# the host sin's argument buffer per round trip (pRotatE three-call form);
# KGE_SIN_CHUNK_BYTES overrides it (tests force several chunks)
SIN_CHUNK_BYTES = int(os.environ.get("KGE_SIN_CHUNK_BYTES", 256 << 20))


def _pinned(n: int, dtype, cache: dict, key: str) -> torch.Tensor:
    """A pinned host buffer of at least n elements, kept for the next call."""
    buf = cache.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 1024), dtype=dtype, pin_memory=True)
        cache[key] = buf
    return buf[:n]


def _rank_protate_library_sin(lib, desc, mode_id, q, nq, off, ids, ranks, ties, lst, flags, ws, st, dev):
    """pRotatE ranks bit-exact to the reference (kge_hip.h: the three-call
    form): the device lists each query's near-ties and decides every one
    whose score interval — under any sin within one ulp of the exact value —
    clears the true score's; only the undecided ones (and their query's true
    entity) go to the host, whose sin is the reference's own call.  Per call:
    one read-back of the undecided counts, then per chunk of ≤
    SIN_CHUNK_BYTES of arguments a pinned device → host copy, the host sin and
    a pinned host → device copy (queries outside the chunk get 0 items)."""
    cnt = torch.empty(nq, dtype=torch.int32, device=dev)
    wsp, wsn, err, s = ws.data_ptr(), ws.numel(), st.err.data_ptr(), _stream(dev)
    _lib.check(lib.kge_rank_filtered_ex(desc, mode_id, q.data_ptr(), nq, off.data_ptr(), ids.data_ptr(),
                                        ranks.data_ptr(), ties.data_ptr(), cnt.data_ptr(),
                                        flags | _lib.RANK_STAGE_LIST, wsp, wsn, err, s),
               "kge_rank_filtered_ex (list)")
    cache = st.__dict__.setdefault("_sin_bufs", {})
    c_host = _pinned(nq, torch.int32, cache, "cnt")
    c_host.copy_(cnt, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()  # the counts size the argument buffers
    c = c_host.numpy().astype(np.int64)
    # a query with more undecided candidates than a list (degenerate tables:
    # > RANK_LIST_CAP near-identical rows) was ranked by the list stage on the
    # device with correctly rounded sin, not the reference's library sin:
    # counted, reported by the caller (KGEModel.rank_device_sin_queries) and logged
    n_dev = int((c > _lib.RANK_LIST_CAP).sum())
    st.__dict__["device_sin_queries"] = st.__dict__.get("device_sin_queries", 0) + n_dev
    if n_dev:
        import logging
        logging.warning("pRotatE ranking: %d of %d queries had more than %d candidates within one ulp of the true "
                        "score under any sin; they were ranked with correctly rounded sin on the device, not the "
                        "reference's library sin", n_dev, nq, _lib.RANK_LIST_CAP)
    items = np.where((c >= 1) & (c <= _lib.RANK_LIST_CAP), 1 + c, 0)
    K = int(desc.entity_dim)
    per_q = items * K * 4
    # chunks of consecutive queries with ≤ SIN_CHUNK_BYTES of arguments each
    bounds, start, acc = [], 0, 0
    for qi in np.nonzero(items)[0]:
        if acc and acc + per_q[qi] > SIN_CHUNK_BYTES:
            bounds.append((start, int(qi)))
            start, acc = int(qi), 0
        acc += int(per_q[qi])
    bounds.append((start, nq))
    for lo, hi in bounds:
        part = np.zeros(nq, dtype=np.int64)
        part[lo:hi] = items[lo:hi]
        item_off = np.zeros(nq + 1, dtype=np.int64)
        np.cumsum(part, out=item_off[1:])
        total = int(item_off[-1])
        off_d = torch.from_numpy(item_off).to(dev)
        args = torch.empty((max(total, 1), K), dtype=torch.float32, device=dev)
        if total:
            _lib.check(lib.kge_rank_sin_args(desc, mode_id, nq, off_d.data_ptr(), args.data_ptr(), wsp, wsn, err, s),
                       "kge_rank_sin_args")
            a_host = _pinned(total * K, torch.float32, cache, "args").view(total, K)
            a_host.copy_(args[:total], non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            s_host = _pinned(total * K, torch.float32, cache, "sins").view(total, K)
            torch.sin(a_host, out=s_host)  # the reference's own call (reference_sin)
            args[:total].copy_(s_host, non_blocking=True)  # the sin values, in place of their arguments
        # (the pinned buffers are reused only after this call's copies: the
        # next chunk synchronises before it writes them)
        _lib.check(lib.kge_rank_finish_sin(desc, mode_id, nq, off_d.data_ptr(), args.data_ptr(), ranks.data_ptr(),
                                           ties.data_ptr(), _ptr(lst), wsp, wsn, err, s),
                   "kge_rank_finish_sin")
    torch.cuda.current_stream(dev).synchronize()  # the pinned buffers are free for the next call


def sample_negatives(triples: torch.Tensor, batch: torch.Tensor, nentity: int, negative_sample_size: int,
                     true_off: torch.Tensor, true_len: torch.Tensor, true_ids: torch.Tensor, weights: torch.Tensor,
                     key: int, max_draws: int, pos_out: torch.Tensor, neg_out: torch.Tensor, w_out: torch.Tensor):
    """One batch of TrainDataset samples on the device (dataloader.py:34-66); see kge_sample_negatives."""
    dev = _require_device(triples, batch, true_off, true_len, true_ids, weights, pos_out, neg_out, w_out)
    B = batch.shape[0]
    assert pos_out.shape == (B, 3) and neg_out.shape == (B, negative_sample_size) and w_out.shape == (B,)
    for t, dt in ((triples, torch.int64), (batch, torch.int64), (true_off, torch.int64), (true_len, torch.int32),
                  (true_ids, torch.int64), (weights, torch.float32), (pos_out, torch.int64),
                  (neg_out, torch.int64), (w_out, torch.float32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError(f"sample_negatives: expected a contiguous {dt} tensor, got {t.dtype}")
    lib = _lib.load()
    _lib.check(lib.kge_sample_negatives(triples.data_ptr(), triples.shape[0], batch.data_ptr(), B, int(nentity),
                                        int(negative_sample_size), true_off.data_ptr(), true_len.data_ptr(),
                                        true_ids.data_ptr(), weights.data_ptr(), int(key) & (2 ** 64 - 1),
                                        int(max_draws), pos_out.data_ptr(), neg_out.data_ptr(), w_out.data_ptr(),
                                        state(dev).err.data_ptr(), _stream(dev)), "kge_sample_negatives")
