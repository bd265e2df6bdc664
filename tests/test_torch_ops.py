"""torch.ops.kge.* — the operator library SURVEY §8(b) names, registered in
C++ (TORCH_LIBRARY(kge, m), csrc/torch/kge_torch_ops.cpp, libkge_torch.so).
CPU: the schemas are registered and the Meta kernels give the right output
metadata, so torch.compile / fake-tensor tracing can carry the ops without
running them; argument errors raise the reference's ValueErrors and CPU
tensors are refused (no CPU path).  The GPU half is tests/test_torch_ops_gpu.py."""
import os

import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from knowledgegraphembedding_amd.torch_ops import LIB_PATH, MODE_IDS, MODEL_IDS  # (loads libkge_torch.so)

TAIL, HEAD, SINGLE = MODE_IDS["tail-batch"], MODE_IDS["head-batch"], MODE_IDS["single"]
ROTATE = MODEL_IDS["RotatE"]


def test_registered_from_the_cpp_library():
    """The ops come from libkge_torch.so's TORCH_LIBRARY, not from Python."""
    assert LIB_PATH.name == "libkge_torch.so" and LIB_PATH.exists()
    assert str(LIB_PATH) in torch.ops.loaded_libraries
    for key in ("CUDA", "Meta", "CPU"):
        assert torch._C._dispatch_has_kernel_for_dispatch_key("kge::score", key), key
    assert torch._C._dispatch_has_kernel_for_dispatch_key("kge::score", "Autograd")


def test_ops_registered_with_schemas():
    for name in ("score", "score_backward", "train_step_grads", "rank_filtered", "sample_negatives"):
        op = getattr(torch.ops.kge, name)
        assert str(op.default._schema).startswith(f"kge::{name}(")
    assert "Tensor? neg" in str(torch.ops.kge.score.default._schema)


def test_fake_shapes():
    with FakeTensorMode():
        ent, rel = torch.empty(100, 32), torch.empty(7, 16)
        pos, neg = torch.empty(8, 3, dtype=torch.int64), torch.empty(8, 20, dtype=torch.int64)
        s = torch.ops.kge.score(ent, rel, pos, neg, TAIL, ROTATE, 12.0, 0.875, None)
        assert s.shape == (8, 20) and s.dtype == torch.float32
        s1 = torch.ops.kge.score(ent, rel, pos, None, SINGLE, ROTATE, 12.0, 0.875, None)
        assert s1.shape == (8, 1)
        l, ge, gr, gm = torch.ops.kge.train_step_grads(ent, rel, None, pos, neg, torch.empty(8), HEAD,
                                                       ROTATE, 12.0, 0.875, True, 1.0, False, 0.0)
        assert l.shape == (4,) and ge.shape == ent.shape and gr.shape == rel.shape and gm.numel() == 0
        r, t = torch.ops.kge.rank_filtered(ent, rel, None, pos, torch.empty(9, dtype=torch.int64),
                                           torch.empty(0, dtype=torch.int64), TAIL, ROTATE, 12.0, 0.875)
        assert r.shape == (8,) and r.dtype == torch.int64 and t.dtype == torch.int32


def test_reference_errors_and_no_cpu_path():
    ent, rel = torch.zeros(10, 8), torch.zeros(3, 4)
    pos, neg = torch.zeros(2, 3, dtype=torch.int64), torch.zeros(2, 5, dtype=torch.int64)
    with pytest.raises(ValueError, match="model 7 not supported"):
        torch.ops.kge.score(ent, rel, pos, neg, TAIL, 7, 12.0, 0.5, None)
    with pytest.raises(ValueError, match="mode 9 not supported"):
        torch.ops.kge.score(ent, rel, pos, neg, 9, ROTATE, 12.0, 0.5, None)
    with pytest.raises(ValueError, match="mode single not supported"):  # training is head-/tail-batch only
        torch.ops.kge.train_step_grads(ent, rel, None, pos, neg, torch.zeros(2), SINGLE, ROTATE, 12.0, 0.5,
                                       True, 1.0, False, 0.0)
    with pytest.raises(RuntimeError, match="ROCm"):
        torch.ops.kge.score(ent, rel, pos, neg, TAIL, ROTATE, 12.0, 0.5, None)
    with pytest.raises(RuntimeError, match="ROCm"):
        torch.ops.kge.rank_filtered(ent, rel, None, pos, torch.zeros(3, dtype=torch.int64),
                                    torch.zeros(0, dtype=torch.int64), TAIL, ROTATE, 12.0, 0.5)


def test_unbuilt_checkout_imports_and_fails_loudly_at_first_op():
    """A checkout without the built libraries must still import (build.py
    imports the package to build it), and the first op must raise — there is
    no CPU or Python fallback."""
    import subprocess
    import sys
    code = (
        "import torch\n"
        "import knowledgegraphembedding_amd as k\n"
        "from knowledgegraphembedding_amd import torch_ops, _lib\n"
        "try:\n"
        "    torch_ops.load()\n"
        "except RuntimeError as e:\n"
        "    assert 'missing' in str(e)\n"
        "else:\n"
        "    raise SystemExit('torch_ops.load() did not raise')\n"
        "try:\n"
        "    _lib.load()\n"
        "except RuntimeError as e:\n"
        "    assert 'missing' in str(e)\n"
        "else:\n"
        "    raise SystemExit('_lib.load() did not raise')\n"
        "print('ok')\n")
    env = dict(os.environ, KGE_TORCH_LIB="/nonexistent/libkge_torch.so", KGE_HIP_LIB="/nonexistent/libkge_hip.so")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
