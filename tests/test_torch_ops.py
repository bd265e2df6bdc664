"""torch.ops.kge.* (knowledgegraphembedding_amd/torch_ops.py): the operator
library SURVEY §8(b) names.  CPU: the schemas are registered and the fake
(meta) implementations give the right output metadata, so torch.compile /
fake-tensor tracing can carry the ops without running them; argument errors
raise the reference's ValueErrors and CPU tensors are refused (no CPU path).
The GPU half is tests/test_torch_ops_gpu.py."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import knowledgegraphembedding_amd.torch_ops  # noqa: F401  (registers the ops)


def test_ops_registered_with_schemas():
    for name in ("score", "score_backward", "train_step_grads", "rank_filtered", "sample_negatives"):
        op = getattr(torch.ops.kge, name)
        assert str(op.default._schema).startswith(f"kge::{name}(")
    assert "Tensor? neg" in str(torch.ops.kge.score.default._schema)


def test_fake_shapes():
    with FakeTensorMode():
        ent, rel = torch.empty(100, 32), torch.empty(7, 16)
        pos, neg = torch.empty(8, 3, dtype=torch.int64), torch.empty(8, 20, dtype=torch.int64)
        s = torch.ops.kge.score(ent, rel, pos, neg, "tail-batch", "RotatE", 12.0, 0.875, None)
        assert s.shape == (8, 20) and s.dtype == torch.float32
        s1 = torch.ops.kge.score(ent, rel, pos, None, "single", "RotatE", 12.0, 0.875, None)
        assert s1.shape == (8, 1)
        l, ge, gr, gm = torch.ops.kge.train_step_grads(ent, rel, None, pos, neg, torch.empty(8), "head-batch",
                                                       "RotatE", 12.0, 0.875, True, 1.0, False, 0.0)
        assert l.shape == (4,) and ge.shape == ent.shape and gr.shape == rel.shape and gm.numel() == 0
        r, t = torch.ops.kge.rank_filtered(ent, rel, None, pos, torch.empty(9, dtype=torch.int64),
                                           torch.empty(0, dtype=torch.int64), "tail-batch", "RotatE", 12.0, 0.875)
        assert r.shape == (8,) and r.dtype == torch.int64 and t.dtype == torch.int32


def test_reference_errors_and_no_cpu_path():
    ent, rel = torch.zeros(10, 8), torch.zeros(3, 4)
    pos, neg = torch.zeros(2, 3, dtype=torch.int64), torch.zeros(2, 5, dtype=torch.int64)
    with pytest.raises(ValueError, match="model Foo not supported"):
        torch.ops.kge.score(ent, rel, pos, neg, "tail-batch", "Foo", 12.0, 0.5, None)
    with pytest.raises(ValueError, match="mode bad not supported"):
        torch.ops.kge.score(ent, rel, pos, neg, "bad", "RotatE", 12.0, 0.5, None)
    with pytest.raises(RuntimeError, match="ROCm"):
        torch.ops.kge.score(ent, rel, pos, neg, "tail-batch", "RotatE", 12.0, 0.5, None)
