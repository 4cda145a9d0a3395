"""Multi-GPU product path: vcap.dist.caption_sharded run by 2 fresh child ranks
(one process per rank, gloo, both on the box's one GPU) gives the single-process reference ids.
tiny_prompt has B = 3 videos: shards of 2 and 1 exercise the padded gather."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from helpers import golden, pad_rows
from vcap.model import trim_generated  # noqa: F401  (import check)

pytestmark = pytest.mark.gpu
HERE = Path(__file__).resolve().parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name", ["tiny_prompt", "tiny"])
def test_caption_sharded_two_ranks_match_goldens(tmp_path, name):
    out = tmp_path / "ids.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(HERE / "dist_worker.py"), name, str(out)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("a rank hung")
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-3000:] for l in logs)
    res = json.loads(out.read_text())
    meta, g = golden(name)
    got = np.array(res["ids"], dtype=np.int32)
    exp = g["hf_greedy_ids"]
    eos = 50256 if meta["gpt2"] == "gpt2" else 1023
    # generate_ids is EOS-padded to max_new; the golden stops where every row has finished
    assert res["world"] == 2 and got.shape[0] == meta["B"]
    assert np.array_equal(got[:, :exp.shape[1]], exp)
    assert (got[:, exp.shape[1]:] == eos).all()


def test_caption_sharded_rccl_one_rank(tmp_path):
    """The RCCL branch of vcap.dist.gather_ids ("nccl" backend: all_gather_into_tensor on the
    device) executed for real: one rank per GPU on this one-GPU box, world size 1; the ids equal
    the reference's goldens."""
    name = "tiny_prompt"
    out = tmp_path / "ids.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(HERE / "dist_worker.py"), name, str(out), "nccl"], env=env,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    res = json.loads(out.read_text())
    meta, g = golden(name)
    got = np.array(res["ids"], dtype=np.int32)
    exp = g["hf_greedy_ids"]
    assert res["world"] == 1 and np.array_equal(got[:, :exp.shape[1]], exp)


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_bench_two_ranks_gloo(tmp_path, device, launcher):
    """The N>1 bench path (one process per rank, sharded videos, decode-lane id copies, ONE
    end-of-run all-gather, MAX-over-ranks timing) rehearsed with 2 ranks sharing the box's GPU
    over gloo (VCAP_BENCH_DIST_BACKEND), started either by `python bench.py --gpus 2` itself (no
    torchrun: the driver's command shape) or by torchrun: rank 0 prints one JSON line for
    n_gpus = 2, and the ids it gathered are, for every timed batch of every rank, the ids a
    single-process serial bf16 run computes on that rank's frames (bench.py seeds rank r's
    videos with 1000 + r)."""
    import torch
    from vcap import configs, prng, weights
    from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder
    steps = 4
    dump = tmp_path / "ids.npy"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["VCAP_BENCH_DIST_BACKEND"] = "gloo"
    run = ([sys.executable] if launcher == "self" else
           [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}"])
    cmd = run + [str(HERE.parent / "bench.py"), "--gpus", "2",
                 "--steps", str(steps), "--warmup", "2", "--cpu-baseline-s", "0", "--no-parity", "--no-decode-alone",
                 "--host-e2e", "0", "--strict-steps", "2", "--dump-ids", str(dump)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["global_batch"] == 16
    assert d["launch"]["world_size"] == 2 and d["launch"]["backend"] == "gloo"
    assert d["launch"]["launcher"].startswith("bench.py --gpus" if launcher == "self" else "external")
    assert d["strict_batch"]["value"] > 0
    got = np.load(dump)
    assert got.shape == (2 * steps, 8, 24)
    va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
    sd = weights.synthetic_state_dict(1, va, ga)
    enc, pre = HipViTEncoder(sd, va, "bf16", device), HipPrefix(sd, ga.n_embd, device=device)
    dec = HipGPT2Decoder(sd, ga, "bf16", device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    cfg.max_blocks = 96
    for rank in range(2):
        video = torch.from_numpy(prng.imagenet_frames(1000 + rank, (8, 16, 3, va.image, va.image))).to(device)
        _, prefix = enc.encode(video, pre)
        exp = dec.generate_ids(prefix, [ga.bos_token_id], cfg).cpu().numpy()
        for t in range(steps):
            assert np.array_equal(got[rank * steps + t], exp), (rank, t)
