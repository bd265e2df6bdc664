"""run.py end to end on the GPU (the reference CLI, run.py:159-342): a tiny
synthetic dataset in the reference's on-disk format, trained with the device
sampler, checkpointed, resumed with -init for a test pass, and the saved
checkpoint/config/.npy files in the reference layout (run.py:93-120)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import spawn_ranks
from knowledgegraphembedding_amd import run, synth

pytestmark = pytest.mark.gpu


def _dataset(root, E=40, R=3, ntrain=300):
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "entities.dict"), "w") as f:
        f.writelines(f"{i}\te{i}\n" for i in range(E))
    with open(os.path.join(root, "relations.dict"), "w") as f:
        f.writelines(f"{i}\tr{i}\n" for i in range(R))
    tr = np.stack([synth.randint(1, (400,), E), synth.randint(2, (400,), R), synth.randint(3, (400,), E)], 1)
    for name, part in (("train.txt", tr[:ntrain]), ("valid.txt", tr[ntrain:ntrain + 50]),
                       ("test.txt", tr[ntrain + 50:])):
        with open(os.path.join(root, name), "w") as f:
            f.writelines(f"e{h}\tr{r}\te{t}\n" for h, r, t in part.tolist())


def _metrics(log_file, prefix):
    """{metric: value} from the reference-format log lines '<prefix><metric> at step <s>: <v>'."""
    out = {}
    for line in open(log_file):
        msg = line.split("INFO", 1)[-1].strip()
        if msg.startswith(prefix):
            k, v = msg[len(prefix):].split(" at step ")
            out[k.strip()] = float(v.split(":")[1])
    return out


def test_run_train_checkpoint_resume(tmp_path):
    data, save = str(tmp_path / "data"), str(tmp_path / "save")
    _dataset(data)
    torch.manual_seed(0)
    args = run.parse_args(["--cuda", "--do_train", "--do_valid", "--do_test", "--device_sampler", "--data_path", data,
                           "--model", "RotatE", "-de", "-n", "16", "-b", "32", "-d", "16", "-g", "6.0", "-adv",
                           "-lr", "0.01", "--max_steps", "30", "--valid_steps", "20", "--log_steps", "10",
                           "--save_checkpoint_steps", "20", "--test_batch_size", "8", "-save", save, "-cpu", "1"])
    run.main(args)
    for f in ("checkpoint", "config.json", "entity_embedding.npy", "relation_embedding.npy"):
        assert os.path.exists(os.path.join(save, f)), f
    test1 = _metrics(os.path.join(save, "train.log"), "Test ")
    assert set(test1) == {"MRR", "MR", "HITS@1", "HITS@3", "HITS@10"}
    assert 0 < test1["MRR"] <= 1 and test1["MR"] >= 1
    cfg = json.load(open(os.path.join(save, "config.json")))
    assert cfg["model"] == "RotatE" and cfg["hidden_dim"] == 16 and cfg["double_entity_embedding"]
    ckpt = torch.load(os.path.join(save, "checkpoint"), map_location="cpu", weights_only=True)
    assert ckpt["step"] == 29
    np.testing.assert_array_equal(np.load(os.path.join(save, "entity_embedding.npy")),
                                  ckpt["model_state_dict"]["entity_embedding"].numpy())
    # resume: -init restores the trained model; its test metrics equal the first run's
    args2 = run.parse_args(["--cuda", "--do_test", "-init", save, "--test_batch_size", "8", "-cpu", "1"])
    run.main(args2)
    test2 = _metrics(os.path.join(save, "test.log"), "Test ")
    for k in test1:
        assert test2[k] == pytest.approx(test1[k], rel=0, abs=1e-12), k


def test_run_countries_config1_vs_reference_cli(tmp_path, golden_info):
    """BASELINE config 1 through run.py: TransE on countries_S1 (the dataset
    files the reference ships, copied to tests/golden/countries_S1), d = 128,
    b = 128, n = 32, with the same flags and seeds the reference's own run.py
    was driven with in tests/golden/make_golden.py (gen_countries_run).  The
    seeded DataLoaders draw the same batches, so the logged training averages,
    the valid / test AUC-PR (run.py:197-204 regions, model.py:322-344) and the
    learning-rate decay at step 150 must follow the reference's log; the
    checkpoint directory has the reference's files (run.py:93-120).
    Tolerances: the GPU's fp32 sums differ from the CPU's in the last bits and
    300 Adam steps carry that drift forward (losses 1e-3 relative, AUC-PR
    2e-3 absolute)."""
    from conftest import GOLDEN
    ref = golden_info["countries_run"]
    save = str(tmp_path / "save")
    # in a fresh interpreter, as the reference's own run was (the in-process
    # case, after an RCCL group: test_run_host_workers_after_rccl_group_in_process);
    # the seeds are set in the same order as before run.main
    import subprocess
    import sys
    code = (f"import sys, numpy as np, torch; np.random.seed({ref['np_seed']}); torch.manual_seed({ref['torch_seed']}); "
            "from knowledgegraphembedding_amd import run; run.main(run.parse_args(sys.argv[1:]))")
    cmd = [sys.executable, "-c", code, "--cuda"] + ref["flags"] + ["--data_path", str(GOLDEN / "countries_S1"),
                                                                  "-save", save]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    _check_countries_run(save, ref)


def _check_countries_run(save, ref):
    """The run's checkpoint directory and logged metrics against the log the
    reference's own run.py wrote (tests/golden/make_golden.py gen_countries_run)."""
    from conftest import GOLDEN
    assert sorted(os.listdir(save)) == ref["files"]
    got = {}
    for line in open(os.path.join(save, "train.log")):
        msg = line.split("INFO", 1)[-1].strip()
        for kind in ("Training average", "Valid", "Test"):
            if msg.startswith(kind + " "):
                k, v = msg[len(kind) + 1:].split(" at step ")
                step, val = v.split(":")
                got[(kind, k.strip(), int(step))] = float(val)
    assert len(got) == len(ref["logs"])
    for kind, metric, step, val in ref["logs"]:
        g = got[(kind, metric, step)]
        tol = 2e-3 if metric == "auc_pr" else 1e-3 * max(1.0, abs(val))
        assert abs(g - val) <= tol, (kind, metric, step, g, val)
    ckpt = torch.load(os.path.join(save, "checkpoint"), map_location="cpu", weights_only=True)
    ref_ckpt = torch.load(str(GOLDEN / "ref_ckpt" / "checkpoint"), map_location="cpu", weights_only=True)
    assert set(ckpt) == set(ref_ckpt)
    assert set(ckpt["model_state_dict"]) == set(ref_ckpt["model_state_dict"])
    assert ckpt["model_state_dict"]["entity_embedding"].shape == (271, 128)


def test_run_host_workers_after_rccl_group_in_process(tmp_path, golden_info):
    """run.py --do_train with host DataLoader workers inside
    the long-lived test process AFTER an RCCL group has been created, used and
    destroyed in it — the round-4 hang's setting.  The workers
    start from run.worker_context()'s forkserver, never as forks of this
    process; BASELINE config 1 (countries_S1, the reference CLI's flags and
    seeds, 300 steps = dozens of worker restarts across epochs) must finish and
    log the reference's metrics, so the start method changed no batch."""
    import socket

    import torch.distributed as dist
    from conftest import GOLDEN
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    t = torch.arange(7, dtype=torch.float32, device=dev)
    dist.all_reduce(t, async_op=True).wait()
    assert dist.get_backend() == "nccl" and torch.equal(t.cpu(), torch.arange(7, dtype=torch.float32))
    dist.destroy_process_group()
    ref = golden_info["countries_run"]
    save = str(tmp_path / "save")
    np.random.seed(ref["np_seed"])
    torch.manual_seed(ref["torch_seed"])
    args = run.parse_args(["--cuda"] + ref["flags"] + ["--data_path", str(GOLDEN / "countries_S1"), "-save", save])
    assert not args.device_sampler and args.do_train
    run.main(args)
    from multiprocessing import forkserver
    assert run.WORKER_START_METHOD == "forkserver" and forkserver._forkserver._forkserver_pid is not None
    _check_countries_run(save, ref)


def _run_rowpart_worker(rank, world, port, data, save, extra=("--device_sampler", "--row_partition")):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0", KGE_PART_EXCHANGE="queries")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    args = run.parse_args(["--cuda", "--do_train", "--do_valid", "--do_test"] + list(extra) +
                          ["--data_path", data, "--model", "RotatE", "-de", "-n", "16", "-b", "32", "-d", "16",
                           "-g", "6.0", "-adv", "-lr", "0.01", "--max_steps", "30", "--valid_steps", "20",
                           "--log_steps", "10", "--save_checkpoint_steps", "20", "--test_batch_size", "8",
                           "-save", save, "-cpu", "1"])
    run.main(args)
    dist.destroy_process_group()


def test_run_data_parallel_host_loader_odd_train_set(tmp_path):
    """run.py data parallel over 2 ranks (gloo, both on cuda:0; the default
    factor exchange) with the CPU DataLoader path and an ODD train set of
    301 triples: the ranks' shards are equal-length (RankShardSampler), so
    their batches keep the same size across the epoch boundaries the 30 steps
    cross, as the exchange's all-gathers require."""
    import socket
    import torch.multiprocessing as mp
    data, save = str(tmp_path / "data"), str(tmp_path / "save")
    _dataset(data, ntrain=301)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    spawn_ranks(_run_rowpart_worker, (2, port, data, save, ()), 2)
    ckpt = torch.load(os.path.join(save, "checkpoint"), map_location="cpu", weights_only=True)
    assert ckpt["step"] == 29
    test1 = _metrics(os.path.join(save, "train.log"), "Test ")
    assert set(test1) == {"MRR", "MR", "HITS@1", "HITS@3", "HITS@10"}


def test_run_row_partition_query_shipping(tmp_path):
    """--row_partition with KGE_PART_EXCHANGE=queries over 2 ranks (gloo, both
    on cuda:0): each rank trains holding only its shard; checkpoints and the
    valid/test passes gather the table (partition.materialize) — the saved
    table has the full shape and a -init test pass reproduces rank 0's logged
    test metrics."""
    import socket
    import torch.multiprocessing as mp
    data, save = str(tmp_path / "data"), str(tmp_path / "save")
    _dataset(data, E=41)  # an odd entity count: the second shard is one row short
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    spawn_ranks(_run_rowpart_worker, (2, port, data, save), 2)
    ckpt = torch.load(os.path.join(save, "checkpoint"), map_location="cpu", weights_only=True)
    assert ckpt["step"] == 29
    assert ckpt["model_state_dict"]["entity_embedding"].shape == (41, 32)
    assert ckpt["optimizer_state_dict"]["state"][0]["exp_avg"].shape == (41, 32)
    test1 = _metrics(os.path.join(save, "train.log"), "Test ")
    assert set(test1) == {"MRR", "MR", "HITS@1", "HITS@3", "HITS@10"}
    args2 = run.parse_args(["--cuda", "--do_test", "-init", save, "--test_batch_size", "8", "-cpu", "1"])
    run.main(args2)
    test2 = _metrics(os.path.join(save, "test.log"), "Test ")
    for k in test1:
        assert test2[k] == pytest.approx(test1[k], rel=0, abs=1e-12), k
