#!/usr/bin/env python3
"""Benchmark: captions/s (+ p50 encode+decode latency) for 16-frame ViT-B/16 -> GPT-2-small.

BASELINE.json `metric`, quoted on configs[1]: batch=8 synthetic 16x3x224x224 videos, bf16,
greedy decode on one MI355X.  One "step" = one pass of the hot path over one batch with the
frames already resident in HBM: fused ViT encode + engine prefix + mapper (vcap_vit_encode),
then the whole 24-token greedy decode with the reference generate()'s processors
(repetition_penalty 1.1, no_repeat_ngram 3, min_new_tokens 8; text_decoder.py:131-144) as
one replayed hipGraph (vcap_gpt2_generate).  For N>1 (torchrun, one rank per GPU) every rank
encodes + decodes its own 8 videos (weak scaling, configs[2]); each batch's int32 token ids are
copied into a per-run buffer on their decode lane, and the buffer is gathered to every rank with
ONE RCCL all_gather_into_tensor at the end of the timed region - the only collective.  (A
collective per batch, issued from the decode lanes, hands work between the lanes and RCCL's
stream and serialised the two-lane pipeline in a one-GPU rehearsal:
profiles/r01_gather_topology.txt.)

Rank 0 prints ONE JSON line.  `roofline` is priced on the dominant kernel (the ViT fc1 GEMM,
`vcap_gemm_kernel<bf16,bf16,1>`), timed live with HIP events around each of its launches in
the timed region (vcap_probe_*).  `cpu_baseline` times the CPU oracle (fp32 torch restatement
of the reference path, oracle/vcap_oracle.py) on a bounded sample on the host cores (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
sys.path.insert(0, str(ROOT))

METRIC = "captions/sec + p50 encode+decode latency, 16-frame ViT-B/16 → GPT-2-small, 1/2/4/8 GPU"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0    # dense block-scaled fp8 MFMA (2x bf16 per clock)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 60 batches: the timed region starts with an empty pipeline and ends with the last decode
    # running alone (~9 ms), so short runs under-report the steady-state rate (30 -> 60 steps:
    # 1207 -> 1230 captions/s, profiles/r02_pipeline_sweeps.txt); 60 steps take ~0.4 s
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8, help="videos per GPU")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--max-new", type=int, default=24)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="fp8: MXFP8 ViT QKV/fc1/fc2 GEMMs (BASELINE configs[4]); the decoder stays bf16")
    ap.add_argument("--dec-precision", default="auto", choices=["auto", "bf16", "fp32"],
                    help="GPT-2 decoder arithmetic: auto = bf16 for --precision bf16 / fp8, fp32 for fp32; fp32 with "
                         "--precision bf16 is the reference's own split (ViT under half-precision autocast, "
                         "src/models/video_encoder.py:261-264; the decoder in fp32, text_decoder.py:131-144)")
    ap.add_argument("--lm-screen", default="on", choices=["on", "off"],
                    help="f32 decoder greedy steps: bf16 lm_head screen + exact f32 rescoring of the tokens it "
                         "cannot rule out (on, same ids) or the f32 lm_head (off)")
    ap.add_argument("--mx-gemms", default="qkv,proj,fc1,fc2",
                    help="--precision fp8: the ViT block GEMMs run in MXFP8 (the others bf16)")
    ap.add_argument("--decode", default="hf_greedy", choices=["hf_greedy", "raw_greedy"])
    ap.add_argument("--beams", type=int, default=1,
                    help=">1: device beam search (preset detailed = 4 beams / max_new 40: BASELINE configs[3])")
    ap.add_argument("--vit", default="vit_base_patch16_224")
    ap.add_argument("--gpt2", default="gpt2")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--serial", action="store_true",
                    help="no encode/decode overlap (each step's decode finishes before the next encode starts)")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="CUs the encode stream leaves to the decode stream (CU-masked stream; 0 = none; "
                         "-1 = auto: 32 with two-batch encodes, else 0 - profiles/r02_decode_experiments.txt)")
    ap.add_argument("--decode-blocks", type=int, default=96,
                    help="cap the decode GEMV grids near this many workgroups (0 = whole-chip grids)")
    ap.add_argument("--dec-lanes", type=int, default=0,
                    help="decodes in flight at once (own stream + workspace + graph each); 0 = auto: 3 for beam "
                         "search (configs[3]: +2.3 %%, 4 streams = the box's 4 hardware queues; "
                         "profiles/r03_c3_schedule_sweep.txt), else 2")
    ap.add_argument("--dec-group", type=int, default=2,
                    help="consecutive batches decoded together as one decode of group*batch rows")
    ap.add_argument("--enc-group", type=int, default=0,
                    help="consecutive batches encoded together as one encode (divides --dec-group); 0 = auto: "
                         "2 while a batch holds <= 128 frames (the N = 768 GEMMs of one 8 x 16-frame batch fill "
                         "1.16 rounds of 256 tiles), else 1")
    ap.add_argument("--decode-cus", type=int, default=-1,
                    help="mask the decode lanes to the first N CUs (the reserved ones + N - reserve of the encode's); "
                         "0: unmasked; -1 (auto): 96 for a bf16, 160 for an fp32 greedy decoder beside a CU-reserved "
                         "encode, else 0")
    ap.add_argument("--confine-decode", action="store_true",
                    help="mask the decode streams to the reserved CUs (default: unmasked, high priority)")
    ap.add_argument("--gemm-policy", type=int, default=0, help="vcap_set_gemm_policy value for A/B runs (0 = auto)")
    ap.add_argument("--host-e2e", type=int, default=10,
                    help="iterations of the SURVEY 8(d) latency variant: pinned host frames -> ids on host, "
                         "one batch at a time (0 disables)")
    ap.add_argument("--cpu-baseline-s", type=float, default=20.0, help="CPU oracle time budget (0 disables)")
    ap.add_argument("--no-parity", dest="parity", action="store_false",
                    help="skip the fp32 agreement check of the last timed batch")
    ap.add_argument("--no-decode-alone", dest="decode_alone", action="store_false",
                    help="skip the decode-step-alone measurement")
    ap.add_argument("--token-exact-steps", type=int, default=-1,
                    help="batches timed in the token_exact leg (the same pipeline with the reference's precision "
                         "split: ViT bf16, GPT-2 decoder fp32) next to a bf16 headline; -1 = --steps, 0 disables")
    ap.add_argument("--roctx", action="store_true",
                    help="roctx stage ranges (ViT_Encoder / GPT2_Decoder_Step around the pipeline's launches, "
                         "vcap/trace.py) for rocprofv3 --marker-trace --kernel-rename; off by default")
    ap.add_argument("--strict-steps", type=int, default=40,
                    help="batches timed in the strict_batch leg (one batch of --batch videos per encode and per "
                         "decode, no coalescing; 0 disables)")
    ap.add_argument("--batch-sizes", default="",
                    help="comma list (the reference's --batch-sizes sweep, core/scripts/benchmark_baseline.py:"
                         "486-493): time the default schedule and the strict per-batch schedule at each batch size")
    ap.add_argument("--sweep-steps", type=int, default=24, help="batches timed per --batch-sizes point")
    ap.add_argument("--dump-ids", default="",
                    help="rank 0 saves every timed batch's ids (gathered over ranks: [world*steps, B, max_new]) "
                         "to this .npy path")
    # the reference harness's exports (core/scripts/benchmark_baseline.py:394-454, flags :517-518)
    ap.add_argument("--export-csv", default="",
                    help="per-iteration CSV of the timed batches (the reference's export_iteration_csv columns); "
                         "with --batch-sizes: the batch-size comparison CSV (export_bs_comparison_csv)")
    ap.add_argument("--export-json", default="", help="summary JSON (the reference's export_summary_json payload)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher check only: every rank joins the process group (gloo), barriers, gathers its "
                         "rank and exits; no GPU work (tests/test_cpu_bench_launch.py)")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------
# --gpus N: one process per GPU.  Under torchrun (WORLD_SIZE set) the ranks already exist and N
# must equal WORLD_SIZE; without it bench.py starts the N ranks itself as child processes BEFORE
# anything touches the GPU (counting devices does not initialise HIP on this image), exits with
# the worst child status, and only rank 0 prints the JSON line.  Flag shape: the reference
# harness's single-command interface (core/scripts/benchmark_baseline.py:500-519) + BASELINE.json's
# "1/2/4/8 GPU".
# ---------------------------------------------------------------------------------------------
REHEARSAL_ENV = "VCAP_BENCH_DIST_BACKEND"   # =gloo: ranks may share the box's GPUs (one-GPU rehearsal)


def _fail(msg: str) -> int:
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    return 2


_GPU_COUNT = []


def _visible_gpus() -> int:
    """GPUs this process may use (HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES
    applied), counted WITHOUT initialising HIP: the parent of self-launched ranks must not touch
    the GPU before it starts them (a process that initialised HIP and then execs / forks children
    that use the GPU is refused on this pool).  torch.cuda.device_count() would fall back to
    torch._C._cuda_getDeviceCount() - a HIP initialisation - whenever amdsmi cannot answer, so the
    amdsmi count is taken directly and a failure refuses the launch instead of falling back."""
    if _GPU_COUNT:
        return _GPU_COUNT[0]
    import torch
    count = getattr(torch.cuda, "_device_count_amdsmi", None)
    if not torch.version.hip or count is None:
        raise RuntimeError("cannot count GPUs without initialising HIP (no ROCm amdsmi device count)")
    n = int(count())
    if n < 0:
        raise RuntimeError("amdsmi could not count the GPUs; refusing to fall back to a HIP initialisation "
                           "in the launcher (set WORLD_SIZE via torchrun, or fix amdsmi)")
    if torch.cuda.is_initialized():
        raise RuntimeError("HIP was initialised while counting GPUs")
    _GPU_COUNT.append(n)
    return n


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_check(args) -> int | None:
    """Validate --gpus against the launch environment.  Returns an exit status to stop with
    (refusal or the self-launched ranks' status), or None to run this process as a rank."""
    n = args.gpus
    if n < 1:
        return _fail(f"--gpus must be >= 1 (got {n})")
    try:
        return _launch_check(args, n)
    except RuntimeError as e:
        return _fail(str(e))


def _launch_check(args, n: int):
    rehearsal = os.environ.get(REHEARSAL_ENV, "nccl") == "gloo"
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != n:
            return _fail(f"--gpus {n} but the launcher started WORLD_SIZE={world} ranks")
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        # this process IS a rank (torchrun started it): it may initialise HIP, so the plain device count
        # (amdsmi, else the HIP runtime's) is the right one here
        import torch
        if not (rehearsal or args.dry_launch) and local_world > torch.cuda.device_count():
            return _fail(f"{local_world} ranks on this node but {torch.cuda.device_count()} visible GPUs "
                         f"(one process per GPU; {REHEARSAL_ENV}=gloo rehearses ranks sharing GPUs)")
        return None
    if n == 1:
        return None
    if not (rehearsal or args.dry_launch) and n > _visible_gpus():
        return _fail(f"--gpus {n} but {_visible_gpus()} visible GPUs "
                     f"(one process per GPU; {REHEARSAL_ENV}=gloo rehearses ranks sharing GPUs)")
    return spawn_ranks(n)


def spawn_ranks(n: int) -> int:
    """Start ranks 0..n-1 of this same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* env, the
    variables torchrun sets), wait for all, and return the worst status: the first failing rank's
    (a rank that fails leaves the others waiting in a collective, so they are then terminated)."""
    import subprocess
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        return _fail("HIP is initialised in the launcher; the ranks must be started before any GPU call")
    env = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), VCAP_BENCH_LAUNCHER="bench.py --gpus (child ranks)")
    cmd = [sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]]
    procs = [subprocess.Popen(cmd, env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    first_bad = 0
    while [p.poll() for p in procs].count(None):      # poll every rank (reaps the dead ones)
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad and not first_bad:
            first_bad = bad[0]
            time.sleep(10)   # let the others report the same failure before they are stopped
            for p in procs:
                if p.poll() is None:
                    p.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
        if p.returncode != 0 and not first_bad:
            first_bad = p.returncode
    return first_bad if first_bad >= 0 else 128 - first_bad


def dry_launch() -> int:
    """--dry-launch: the rendezvous and the collective path of the ranks, on gloo, no GPU."""
    import torch
    import torch.distributed as dist
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
        parts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.tensor([rank], dtype=torch.int64))
        ranks = [int(p.item()) for p in parts]
        dist.destroy_process_group()
    else:
        ranks = [0]
    if rank == 0:
        print(json.dumps({"dry_launch": True, "world_size": world, "ranks": ranks,
                          "launcher": launcher_name()}), flush=True)
    return 0


def launcher_name() -> str:
    if os.environ.get("VCAP_BENCH_LAUNCHER"):
        return os.environ["VCAP_BENCH_LAUNCHER"]
    return "external (torchrun env)" if "WORLD_SIZE" in os.environ else "single process"


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """N = len(os.sched_getaffinity(0)), bounded by the cgroup's CPU quota when one
    is set (the GPU box's affinity lists all 256 host CPUs while its quota is 16; 256 threads on 16
    CPUs of quota only add contention).  Returns (threads used, affinity count, quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(sd, va, ga, frames_np, budget_s: float, max_new: int, beams: int = 1):
    """Time the CPU oracle (fp32 torch restatement of the reference path) on the host cores
    (BASELINE.md §3): B = 1 (the reference's single-clip CPU path) p50 of >= 5
    captions after one warm-up, and B = all the workload's videos (8) p50 of the runs the budget
    allows (>= 1).  `value` is the B = 8 rate (the same batch the GPU line captions; the higher of
    the two).  The B = 8 ids are returned for the parity check of the GPU run (the oracle as the
    checker, never as the thing measured)."""
    import torch
    from oracle import vcap_oracle as O
    threads, aff, quota = cpu_threads()
    torch.set_num_threads(threads)
    prompt = [ga.bos_token_id]

    def run(v):
        t0 = time.perf_counter()
        ids = O.caption_ids(sd, va, ga, torch.from_numpy(v), prompt, max_new_tokens=max_new, num_beams=beams)
        return time.perf_counter() - t0, ids

    t_start = time.perf_counter()
    with torch.no_grad():
        b1 = [run(frames_np[:1])[0] for _ in range(6)]            # 1 warm-up + 5
        B = frames_np.shape[0]
        b8, ids8 = [], None
        while not b8 or (time.perf_counter() - t_start < budget_s and len(b8) < 5):
            t, ids8 = run(frames_np)
            b8.append(t)
    p1, p8 = statistics.median(b1[1:]), statistics.median(b8)
    work = (f"1x{frames_np.shape[1]}x3x{va.image}x{va.image} frames per video, fp32 torch CPU oracle, "
            f"{'HF-greedy' if beams == 1 else f'HF beam {beams}'} max_new {max_new}")
    return {"value": B / p8, "unit": "captions/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "affinity_cores": aff, "cgroup_cpu_quota": quota, "torch_threads": torch.get_num_threads(),
            "sample": f"B={B}: {len(b8)} batch runs, p50 {p8:.2f} s; B=1: 6 single-video captions, p50 of the "
                      f"last 5 = {p1 * 1e3:.0f} ms ({work}); value = the B={B} rate",
            "b1": {"captions_per_s": 1.0 / p1, "p50_latency_ms": p1 * 1e3, "runs": len(b1) - 1},
            "b8": {"videos": B, "captions_per_s": B / p8, "p50_batch_s": p8, "runs": len(b8)},
            "_ids": ids8}


def oracle_agreement(last, ref_ids, eos, beams: int = 1):
    """Captions of the last timed batch against the CPU oracle's on the same frames.  Greedy: HF
    generate's output length (trimmed where every row has finished).  Beam search: each row's best
    hypothesis up to and including its first EOS (the device search and HF pad differently after
    it)."""
    from vcap.model import raw_greedy_tokens, trim_generated
    import torch
    if beams > 1:
        got = raw_greedy_tokens(last, eos)
        exp = raw_greedy_tokens(torch.as_tensor(ref_ids), eos)
    else:
        got = trim_generated(last, eos)
        exp = ref_ids.tolist() if hasattr(ref_ids, "tolist") else ref_ids
    same = sum(int(a == b) for a, b in zip(got, exp))
    return {"against": "CPU oracle (fp32 restatement pinned to the reference's goldens) on the same frames",
            "batch": "last timed batch", "captions": len(exp), "captions_identical": same,
            "first_divergent_step": [next((i for i, (x, y) in enumerate(zip(a, b)) if x != y),
                                          None if len(a) == len(b) else min(len(a), len(b)))
                                     for a, b in zip(got, exp)]}


STRICT_RESERVE = 32   # CUs the strict_batch leg reserves off its encode stream
PMC_FILES = ("r06_pmc.json", "r05_pmc.json", "r04_pmc_colgroup.json", "r04_pmc.json", "r02_pmc.json", "r01_pmc.json")   # newest first


def _pmc_file(M: int):
    """The committed rocprofv3 PMC summary (tools/pmc.sh + tools/pmc_report.py) collected on ViT
    GEMM launches of M rows, or None (PMC counters cannot be read inside bench.py)."""
    for name in PMC_FILES:
        try:
            d = json.loads((ROOT / "profiles" / name).read_text())
        except (OSError, ValueError):
            continue
        if d.get("vit_rows", 25216) == M:
            return name, d
    return None, None


def fc1_traffic(M: int, N: int, K: int):
    """HBM bytes per fc1 launch (FETCH_SIZE x2 + WRITE_SIZE) from the committed PMC passes, when
    they were collected on this exact shape; None otherwise."""
    name, d = _pmc_file(M)
    if d is None or (N, K) != (3072, 768):
        return None
    k = next((v for n, v in d["vit_kernels"].items() if "gemm256_kernel<unsigned short, unsigned short, 1>" in n), None)
    if not k or k.get("fetch_bytes") is None or k.get("write_bytes") is None:
        return None
    return float(k["fetch_bytes"] + k["write_bytes"])


def pmc_summary(vit: str, gpt2: str, M: int, precision: str):
    """MFMA utilisation of the ViT GEMMs and the decode's HBM bytes per token step from the
    committed PMC passes on this configs[1] workload; None for other workloads."""
    if (vit, gpt2, precision) != ("vit_base_patch16_224", "gpt2", "bf16"):
        return None
    name, d = _pmc_file(M)
    if d is None:
        return None
    # (r04 splits the attn-proj / fc2 launches of the shared <bf16, f32, 2> instantiation: "...2>[fc2]")
    util = {k.split("<", 1)[1].replace(">", " ").strip(): round(v["mfma_util"], 3)
            for k, v in d["vit_kernels"].items() if "gemm256" in k and v.get("mfma_util")}
    return {"source": f"profiles/{name} (rocprofv3 --pmc, separate passes, ViT launches of {M} rows)",
            "vit_gemm_mfma_util": util,
            "decode_hbm_bytes_per_token_step": d["decode"]["hbm_bytes_per_token_step"]}


def decode_step_alone(dec, prefix, ids_cfg, ga):
    """Per-token decode step on an otherwise idle GPU: (24-token graph - 1-token graph) / 23, both
    replayed after warm-up (the prefill cancels)."""
    import torch
    from vcap.model import GenConfig
    import dataclasses
    res = {}
    lo = 2 if ids_cfg.num_beams > 1 else 1
    for mx in (lo, ids_cfg.max_new_tokens):
        cfg = dataclasses.replace(ids_cfg, max_new_tokens=mx, use_graph=True, max_blocks=0)
        out = torch.empty(prefix.shape[0], mx, dtype=torch.int32, device=prefix.device)
        for _ in range(3):
            dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out)
        torch.cuda.synchronize()
        res[mx] = (time.perf_counter() - t) / 20
    return (res[ids_cfg.max_new_tokens] - res[lo]) / (ids_cfg.max_new_tokens - lo), res[lo]


def describe(xs):
    """mean / std / p50 / p99 / min / max (the reference's stage statistics plus p50)."""
    import numpy as np
    a = np.asarray(xs, dtype=np.float64)
    return {"mean": float(a.mean()), "std": float(a.std()), "p50": float(np.median(a)),
            "p99": float(np.percentile(a, 99)), "min": float(a.min()), "max": float(a.max()), "n": int(a.size)}


def launch_summary(launches, rows_main, flops_of, bytes_of=None):
    """Per-launch probe records [(ms, rows)] -> the population of full-group launches (rows_main
    rows) priced with its own FLOPs, plus every other population (a flushed partial group)."""
    from vcap import probe
    pops = probe.by_rows(launches)
    main = pops.get(rows_main) or max(pops.values(), key=len)
    r_main = rows_main if rows_main in pops else max(pops, key=lambda r: len(pops[r]))
    out = {"launches": len(main), "avg_launch_ms": sum(main) / len(main), "flops_per_launch": flops_of(r_main),
           "other_populations": {str(r): {"launches": len(v), "avg_launch_ms": sum(v) / len(v)}
                                 for r, v in pops.items() if r != r_main}}
    if bytes_of is not None:
        out["bytes_per_launch"] = bytes_of(r_main)
    return out


def parity_report(sd, va, ga, video, pre, enc, dec, cfg, last, dev):
    """The benchmarked precision against the fp32 parity mode on the benchmark's own frames.
    Greedy: every divergent caption is explained by the fp32 margin at its first divergent step
    against the tested precision's teacher-forced logit error (vcap.fidelity.greedy_divergence).
    Beam search: the fp32 score of the tested search's best hypothesis against the fp32 search's
    (vcap.fidelity.beam_divergence)."""
    import torch
    from vcap import fidelity
    from vcap.model import HipGPT2Decoder, HipViTEncoder
    enc32 = HipViTEncoder(sd, va, "fp32", dev)
    dec32 = HipGPT2Decoder(sd, ga, "fp32", dev)
    _, pre32 = enc32.encode(video, pre)
    prompt = [ga.bos_token_id]
    L, B = cfg.max_new_tokens, video.shape[0]
    against = "fp32 parity mode on the same frames (token-identical to the reference goldens)"
    if cfg.num_beams > 1:
        ids32 = dec32.generate_ids(pre32, prompt, cfg).cpu()
        rep = fidelity.beam_divergence(dec32, pre32, prompt, last.tolist(), ids32.tolist(), cfg)
        rep.update({"against": against, "batch": "last timed batch"})
        return rep
    logits32 = torch.empty(L, B, ga.vocab, dtype=torch.float32, device=dev)
    ids32 = dec32.generate_ids(pre32, prompt, cfg, out=torch.empty(B, L, dtype=torch.int32, device=dev),
                               logits_out=logits32)
    _, pre_t = enc.encode(video, pre)
    tf = fidelity.teacher_forced_logits(dec, pre_t, prompt, ids32, L)
    rep = fidelity.greedy_divergence(last.numpy(), ids32.cpu().numpy(), logits32, tf, cfg)
    rep.update({"against": against, "batch": "last timed batch",
                "evidence": "tested-precision encoder + decoder teacher-forced along the fp32 tokens; "
                            "fp32_margin = fp32 processed score of its token minus that of the tested "
                            "path's token at the first divergent step"})
    return rep


# Decode lanes masked to the first N CUs (the 32 the encode leaves free + N - 32 of the encode's): the
# decode's workgroups then never land on the other encode CUs between two GEMM workgroups.  Measured
# (profiles/r06_decode_cus_sweep.txt, same box, interleaved): bf16 decoder unmasked 1246.7-1249.1,
# 64 CUs 1268.3-1269.1, 96 CUs 1269.7-1271.8, 128 CUs 1261.8-1264.3, 160 CUs 1258.6-1259.7 captions/s
# (p50 28.4 -> 30.9 ms at 96); fp32 decoder unmasked 1180.7-1181.5, 64 CUs 1016.4-1016.8 (the decode
# becomes the bottleneck), 128 CUs 1176.2-1177.7, 160 CUs 1193.0-1193.1.
DECODE_CUS = {"bf16": 96, "fp32": 160}


def auto_decode_cus(args, dec_precision: str) -> int:
    if args.serial or args.confine_decode or args.reserve_cus <= 0 or args.beams != 1 or args.precision != "bf16":
        return 0
    return DECODE_CUS.get(dec_precision, 0)


def time_schedule(enc, pre, dec, cfg, video, prompt, dev, world, steps, warmup, keep_last=False, **sched):
    """Time `steps` batches of `video` through a fresh CaptionPipeline with the given schedule,
    bracketed like the headline (synchronize + barrier on both sides, max over ranks): captions/s,
    per-batch latency stats (encode start -> ids) and B / p50 (+ the last batch's ids as "_last")."""
    import torch
    import torch.distributed as dist
    from vcap.pipeline import CaptionPipeline
    B = video.shape[0]
    pipe = CaptionPipeline(enc, pre, dec, cfg, B, prompt, dev, **sched)
    try:
        for _ in range(max(warmup, 1)):
            pipe.submit(video)
        pipe.synchronize()
        starts = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
        mids = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(steps):
            pipe.submit(video, starts[k], mids[k], ends[k])
        pipe.synchronize()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
        lat = [s.elapsed_time(e) for s, e in zip(starts, ends)]
        stage = ([s.elapsed_time(m) for s, m in zip(starts, mids)], [m.elapsed_time(e) for m, e in zip(mids, ends)])
        last = pipe.result(pipe.last_slot).cpu() if keep_last else None
    finally:
        pipe.close()
    p50 = statistics.median(lat)
    out = {"value": world * B * steps / elapsed, "ms_per_step": elapsed / steps * 1e3, "steps": steps,
           "p50_latency_ms": p50, "captions_per_s_b_over_p50": world * B / (p50 / 1e3),
           "latency_ms_stats": describe(lat), "_per_batch_ms": (lat, *stage)}
    if keep_last:
        out["_last"] = last
    return out


def export(args, out, B, lat, vit_ms, dec_ms, ids_all, dec_alone, sweep_rows, eos, mem_mb):
    """--export-csv / --export-json in the reference harness's shapes (vcap/report.py;
    core/scripts/benchmark_baseline.py:394-454, 665-738): one batch size -> the per-iteration CSV
    + {env, config, summary, iterations}; a --batch-sizes sweep -> the comparison CSV +
    {env, config, comparison, per_batch_summary, per_batch_iterations}."""
    import torch
    from vcap import report
    ids = ids_all.cpu().numpy()
    lens = [[int((row == eos).argmax()) + 1 if (row == eos).any() else int(row.size) for row in batch]
            for batch in ids]
    previews = ["ids " + " ".join(str(int(t)) for t in batch[0][:lens[k][0]]) for k, batch in enumerate(ids)]
    step_ms = dec_alone["step_us"] / 1e3 if dec_alone else None
    rows = report.iteration_rows(B, lat, vit_ms, dec_ms, lens, previews, step_ms, mem_mb)
    props = torch.cuda.get_device_properties(0)
    env = {"torch": torch.__version__, "torch_hip": torch.version.hip, "device": torch.cuda.get_device_name(0),
           "gcn_arch": getattr(props, "gcnArchName", ""), "total_vram_mb": props.total_memory / 2**20}
    cfg = {"frames": "synthetic (resident in HBM)", "ckpt": "seeded random-init (weights seed 1)", "device": "cuda:0",
           "prompt": "BOS", "warmup": args.warmup, "iters": args.steps, "max_new_tokens": args.max_new,
           "num_frames": args.frames, "image_size": 224, "prefix_len": 4, "ln_scale": 0.6, "in_weight": 0.4,
           "batch_sizes": sorted(sweep_rows) if sweep_rows else [B], "precision": args.precision}
    if sweep_rows:
        summaries = {bs: report.build_summary(r, bs) for bs, r in sweep_rows.items()}
        comp = [report.comparison_row(summaries[bs], args.warmup, args.sweep_steps) for bs in sorted(summaries)]
        if args.export_csv:
            report.export_bs_comparison_csv(args.export_csv, comp)
        if args.export_json:
            report.export_summary_json(args.export_json, {
                "env": env, "config": cfg, "comparison": comp,
                "per_batch_summary": {str(bs): v for bs, v in summaries.items()},
                "per_batch_iterations": {str(bs): v for bs, v in sweep_rows.items()}, "bench_line": out})
        return
    if args.export_csv:
        report.export_iteration_csv(args.export_csv, rows)
    if args.export_json:
        report.export_summary_json(args.export_json, {"env": env, "config": cfg,
                                                      "summary": report.build_summary(rows, B),
                                                      "iterations": rows, "bench_line": out})


def workload_tag(args, world):
    if args.precision == "fp8":
        return "configs[4]-shaped, MXFP8 ViT GEMMs"
    if args.vit == "vit_large_patch14_224" and args.gpt2 == "gpt2-medium" and args.beams > 1:
        return "configs[3]"
    return "configs[1]" + ("/[2]" if world > 1 else "")


def main():
    args = parse()
    rc = launch_check(args)
    if rc is not None:
        sys.exit(rc)
    if args.dry_launch:
        sys.exit(dry_launch())
    import numpy as np
    import torch
    import torch.distributed as dist

    from vcap import configs, prng, probe, weights
    from vcap import _native as N
    from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder
    from vcap.pipeline import CaptionPipeline
    from vcap.dist import gather_ids
    from vcap import report

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VCAP_BENCH_DIST_BACKEND=gloo + ranks sharing GPUs (local % device count): a rehearsal of the
    # N>1 path on a one-GPU box; the driver's multi-GPU runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("VCAP_BENCH_DIST_BACKEND", "nccl")
    gpu = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    if args.dec_lanes <= 0:
        args.dec_lanes = 3 if args.beams > 1 else 2
    if args.enc_group <= 0:
        args.enc_group = 2 if args.batch * args.frames <= 128 and args.dec_group % 2 == 0 else 1
    if args.reserve_cus < 0:
        args.reserve_cus = 32 if args.enc_group == 2 else 0

    va, ga = configs.vit_arch(args.vit), configs.gpt2_arch(args.gpt2)
    sd = weights.synthetic_state_dict(1, va, ga)
    B, T = args.batch, args.frames
    frames_np = prng.imagenet_frames(1000 + rank, (B, T, 3, va.image, va.image))   # distinct videos per rank
    video = torch.from_numpy(frames_np).to(dev)

    N.check(N.lib().vcap_set_gemm_policy(args.gemm_policy), "gemm policy")
    if args.roctx:
        from vcap import trace
        trace.enable()
    mx_gemms = tuple(g for g in args.mx_gemms.split(",") if g)
    enc = HipViTEncoder(sd, va, args.precision, dev, mx_gemms=mx_gemms)
    pre = HipPrefix(sd, ga.n_embd, device=dev)
    if args.dec_precision == "auto":
        args.dec_precision = "fp32" if args.precision == "fp32" else "bf16"
    decode_cus_auto = args.decode_cus < 0
    if decode_cus_auto:
        args.decode_cus = auto_decode_cus(args, args.dec_precision)
    dec = HipGPT2Decoder(sd, ga, args.dec_precision, dev, screen=args.lm_screen == "on")
    if args.decode == "hf_greedy":
        cfg = GenConfig(args.max_new, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, not args.no_graph,
                        num_beams=args.beams)
    else:
        cfg = GenConfig.raw_greedy(args.max_new, ga.eos_token_id, not args.no_graph)
    cfg.max_blocks = 0 if args.serial else args.decode_blocks
    # every timed batch's ids -> row (submission index - timed_base) of a per-run buffer, copied on
    # the decode lane that produced them
    ids_all = torch.zeros(max(args.steps, 1), B, args.max_new, dtype=torch.int32, device=dev)
    timed_base = [1 << 30]

    def keep(ids, first_k):
        for i in range(ids.shape[0] // B):
            t = first_k + i - timed_base[0]
            if 0 <= t < args.steps:
                ids_all[t].copy_(ids[i * B:(i + 1) * B])
        return ids

    pipe = CaptionPipeline(enc, pre, dec, cfg, B, [ga.bos_token_id], dev,
                           gather=keep if (world > 1 or args.dump_ids or args.export_csv or args.export_json)
                           else None,
                           reserve_cus=0 if args.serial else args.reserve_cus,
                           dec_lanes=1 if args.serial else args.dec_lanes,
                           confine_decode=False if args.serial else (args.decode_cus if args.decode_cus > 0
                                                                      else args.confine_decode),
                           dec_group=1 if args.serial else args.dec_group,
                           enc_group=1 if args.serial else args.enc_group)

    def step(t0=None, t1=None, t2=None):
        pipe.submit(video, t0, t1, t2)
        if args.serial:
            pipe.synchronize()

    for _ in range(max(args.warmup, 1)):
        step()
    pipe.synchronize()   # (flushes a partial decode group)
    torch.cuda.synchronize(dev)
    if world > 1:
        gather_ids(ids_all, world)  # communicator set-up outside the timed region
        torch.cuda.synchronize(dev)
        dist.barrier()
    # live per-launch timing of the dominant encode kernels inside the timed region only: enabled
    # here, read (and disabled) right after it, before any other leg launches an encode
    probe_cap = va.depth * (args.steps + 2)
    for site in ("vit.fc1", "vit.attention"):
        probe.enable(site, probe_cap)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    mids = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    timed_base[0] = pipe.k
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(starts[k], mids[k], ends[k])
    pipe.synchronize()   # decodes a trailing partial group too
    if world > 1:
        gathered = gather_ids(ids_all, world)  # [world * steps, B, max_new] on every rank
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    probes = {site: probe.read(site, probe_cap) for site in ("vit.fc1", "vit.attention")}
    E_enc = 1 if args.serial else args.enc_group
    enc_launches = -(-args.steps // E_enc)          # encodes issued in the timed region (a trailing
    expected = enc_launches * (va.depth - 1)        # partial group is flushed inside it)
    for site, launches in probes.items():
        if len(launches) != expected:
            raise RuntimeError(f"probe {site}: {len(launches)} launches in the timed region, expected {expected}")

    # SURVEY 8(d) latency: a host-pinned [B,T,3,H,W] fp32 tensor -> H2D -> encode -> decode ->
    # token ids on the host, one batch at a time (outside the timed throughput region)
    host_lat = []
    if args.host_e2e > 0:
        pinned = torch.from_numpy(frames_np).pin_memory()
        vid_h = torch.empty_like(video)
        for _ in range(args.host_e2e + 1):
            torch.cuda.synchronize(dev)
            t_h = time.perf_counter()
            # H2D on torch's own stream (the pinned-memory allocator records its event there, not on
            # the pipeline's external CU-masked stream that close() destroys); the encode waits on it
            vid_h.copy_(pinned, non_blocking=True)
            pipe.s_enc.wait_stream(torch.cuda.current_stream(dev))
            ids_dev = pipe.result(pipe.submit(vid_h))
            ids_host = (gather_ids(ids_dev, world) if world > 1 else ids_dev).cpu()
            host_lat.append(time.perf_counter() - t_h)
        host_lat = host_lat[1:]
        torch.cuda.synchronize(dev)
        del ids_host, pinned, vid_h

    if args.dump_ids and rank == 0:
        np.save(args.dump_ids, (gathered if world > 1 else ids_all).cpu().numpy())

    # caption lengths of the last timed batch (new tokens up to and including EOS)
    last = pipe.result(pipe.last_slot).cpu()
    pipe.synchronize()
    prompt = [ga.bos_token_id]
    # strict_batch: what a caller with ONE batch of B videos sees - one B-video encode and one B-row
    # decode per batch (no two-batch coalescing), two decode lanes, timed like `value`
    strict = None
    if args.strict_steps > 0 and not args.serial:
        # 32 CUs reserved off the encode stream, as for the coalesced schedule: 1066 vs 928 captions/s
        # and p50 22.1 vs 24.6 ms unreserved (profiles/r04_strict_reserve_sweep.txt)
        strict = time_schedule(enc, pre, dec, cfg, video, prompt, dev, world, args.strict_steps, args.warmup,
                               dec_lanes=args.dec_lanes, dec_group=1, enc_group=1, reserve_cus=STRICT_RESERVE)
        strict["schedule"] = (f"one {B}-video encode + one {B}-row decode graph per batch, {args.dec_lanes} decode "
                              f"lanes, encode stream off {STRICT_RESERVE} CUs, no coalescing")
        strict.pop("_per_batch_ms")
    # token_exact: the same pipeline with the reference's precision split - ViT bf16 (its half-precision
    # autocast, src/models/video_encoder.py:261-264), GPT-2 decoder fp32 (text_decoder.py:131-144) -
    # timed like `value`; its last batch is checked against the CPU oracle below (8 of 8 expected)
    token_exact = None
    te_steps = args.steps if args.token_exact_steps < 0 else args.token_exact_steps
    if (te_steps > 0 and not args.serial and args.precision == "bf16" and args.dec_precision == "bf16"
            and args.beams == 1 and args.decode == "hf_greedy"):
        dec32 = HipGPT2Decoder(sd, ga, "fp32", dev, screen=args.lm_screen == "on")
        token_exact = time_schedule(enc, pre, dec32, cfg, video, prompt, dev, world, te_steps, args.warmup,
                                    keep_last=True, dec_lanes=args.dec_lanes, dec_group=args.dec_group,
                                    enc_group=args.enc_group, reserve_cus=args.reserve_cus,
                                    confine_decode=auto_decode_cus(args, "fp32") if decode_cus_auto
                                    else args.decode_cus)
        lat_t, vit_t, dec_t = token_exact.pop("_per_batch_ms")
        token_exact["stage_ms_p50"] = {"vit_encode_prefix": statistics.median(vit_t),
                                       "prefix_ready_to_ids": statistics.median(dec_t)}
        token_exact["precision"] = "ViT bf16 + GPT-2 decoder fp32 (bf16 lm_head screen + exact f32 rescoring)" \
            if dec32.screen else "ViT bf16 + GPT-2 decoder fp32"
        token_exact["decode_cus"] = auto_decode_cus(args, "fp32") if decode_cus_auto else args.decode_cus
        token_exact["schedule"] = ("the headline's (same lanes, groups, CU reservation and decode grid cap); decode "
                                   f"lanes masked to {token_exact['decode_cus']} CUs" if token_exact["decode_cus"]
                                   else "the headline's (same lanes, groups, CU reservation and decode grid cap)")
        if args.decode_alone:
            with torch.cuda.stream(torch.cuda.Stream(dev)):
                _, pre_a = enc.encode(video, pre)
                step_s, _ = decode_step_alone(dec32, pre_a, cfg, ga)
            token_exact["decode_step_alone_us"] = step_s * 1e6
        del dec32
        torch.cuda.empty_cache()
    sweep = None
    sweep_rows = {}   # batch size -> the default schedule's per-batch rows (reference export shape)
    if args.batch_sizes:
        sweep = []
        for bs in [int(x) for x in args.batch_sizes.split(",") if x]:
            vid = torch.from_numpy(prng.imagenet_frames(2000 + bs, (bs, T, 3, va.image, va.image))).to(dev)
            eg = 2 if bs * T <= 128 and args.dec_group % 2 == 0 else 1
            pt = {"batch": bs}
            pt["default_schedule"] = time_schedule(enc, pre, dec, cfg, vid, prompt, dev, world, args.sweep_steps,
                                                   args.warmup, dec_lanes=args.dec_lanes, dec_group=args.dec_group,
                                                   enc_group=eg, reserve_cus=32 if eg == 2 else 0)
            pt["strict_batch"] = time_schedule(enc, pre, dec, cfg, vid, prompt, dev, world, args.sweep_steps,
                                               args.warmup, dec_lanes=args.dec_lanes, dec_group=1, enc_group=1,
                                               reserve_cus=STRICT_RESERVE)
            lat_b, vit_b, dec_b = pt["default_schedule"]["_per_batch_ms"]
            sweep_rows[bs] = report.iteration_rows(bs, lat_b, vit_b, dec_b, [], [], None,
                                                   torch.cuda.max_memory_allocated(dev) / 2**20)
            for k in ("default_schedule", "strict_batch"):
                pt[k].pop("latency_ms_stats")
                pt[k].pop("_per_batch_ms")
            print(f"sweep batch {bs}: default {pt['default_schedule']['value']:.1f}, strict "
                  f"{pt['strict_batch']['value']:.1f} captions/s", file=sys.stderr, flush=True)
            sweep.append(pt)
            del vid
        torch.cuda.empty_cache()
    # parity of what was timed (outside the timed region): the last batch's ids against the fp32
    # parity mode (token-exact against the reference: tests/test_gpu_parity.py) on the same frames,
    # with the near-tie evidence for every divergent caption (vcap/fidelity.py)
    parity = None
    dec_alone = None
    if (args.precision != "fp32" or args.dec_precision != "fp32") and args.parity:
        parity = parity_report(sd, va, ga, video, pre, enc, dec, cfg, last, dev)
        torch.cuda.empty_cache()
    if args.decode_alone:
        with torch.cuda.stream(torch.cuda.Stream(dev)):
            _, pre_a = enc.encode(video, pre)
            step_s, prefill_s = decode_step_alone(dec, pre_a, cfg, ga)
        wbytes = ga.weight_elems_per_step() * (4 if args.dec_precision == "fp32" else 2)
        dec_alone = {"what": (f"one token step of the B-row greedy decode graph" if args.beams == 1 else
                              f"one step of the device beam search graph ({B} x {args.beams} beams)") +
                             ", alone on the GPU (difference of a max_new-step and a 1-2-step graph)",
                     "step_us": step_s * 1e6, "prefill_plus_one_step_us": prefill_s * 1e6,
                     "weight_bytes_per_step": wbytes, "achieved_gbs": wbytes / step_s / 1e9,
                     "frac_of_hbm_peak": wbytes / step_s / 1e9 / PEAK_HBM_GBS}
    eos = ga.eos_token_id
    lens = [int((row == eos).nonzero()[0, 0]) + 1 if bool((row == eos).any()) else int(row.numel()) for row in last]

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    lat = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    vit_ms = [s.elapsed_time(m) for s, m in zip(starts, mids)]
    dec_ms = [m.elapsed_time(e) for m, e in zip(mids, ends)]

    if rank == 0:
        E = 1 if args.serial else args.enc_group   # batches per encode launch
        M = E * B * T * va.tokens                    # ViT rows per GEMM launch (full encode group)
        peak = {"bf16": PEAK_BF16_TFLOPS, "fp8": PEAK_FP8_TFLOPS}.get(args.precision, PEAK_F32_TFLOPS)
        ab = 2 if args.precision in ("bf16", "fp8") else 4

        def fc1_flops(rows):
            return 2.0 * rows * va.mlp * va.dim

        # where the encode runs the QKV projection and the attention as one kernel
        # (vcap_vit_qkv_attention: bf16 ViT-B/16 and ViT-L/14 frames) the "vit.attention" probe times
        # it; otherwise the probe times the attention kernel alone
        fused_attn = enc.fuses_qkv_attention(0)   # the library's own predicate (every probed block alike)

        def attn_flops(rows):
            core = 4.0 * (rows // va.tokens) * va.heads * va.tokens * va.tokens * 64
            return core + (2.0 * rows * 3 * va.dim * va.dim if fused_attn else 0.0)

        def attn_bytes(rows):
            if fused_attn:   # LayerNorm rows in, attention rows out (q / k / v stay on chip), weights
                return float(2 * rows * va.dim * ab + 3 * va.dim * va.dim * ab)
            return float(rows * 3 * va.dim * ab + rows * va.dim * (1 if args.precision == "fp8" else ab))

        fc1 = launch_summary(probes["vit.fc1"], M, fc1_flops)
        att = launch_summary(probes["vit.attention"], M, attn_flops, attn_bytes)
        achieved = fc1["flops_per_launch"] / (fc1["avg_launch_ms"] / 1e3) / 1e12
        vit_exec = B * T * va.flops_per_frame(cls_tail=True)
        dec_bytes = float(args.max_new * ga.weight_elems_per_step() * (4 if args.dec_precision == "fp32" else 2))
        t_roof = vit_exec / (peak * 1e12) + dec_bytes / (PEAK_HBM_GBS * 1e9)
        total = world * B * args.steps
        value = total / elapsed
        p50 = statistics.median(lat)
        out = {
            "metric": METRIC, "value": value, "unit": "captions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": ({"bf16": "bf16", "fp8": f"mxfp8-e4m3 (ViT {'/'.join(enc.mx_gemms)})"}.get(args.precision, "f32") +
                       ("" if (args.precision == "fp32") == (args.dec_precision == "fp32") and args.precision != "fp8"
                        else f" + {'f32' if args.dec_precision == 'fp32' else 'bf16'} decoder")),
            "data": "synthetic (seeded U[0,1) frames, ImageNet-normalised; seeded random-init weights)",
            "config": {"workload": f"batch={B} synthetic {T}x3x224x224 videos per GPU, {args.vit} + {args.gpt2}, "
                                   f"{args.decode if args.beams == 1 else f'beam-{args.beams}'} decode max_new {args.max_new} "
                                   f"(BASELINE {workload_tag(args, world)})",
                       "num_beams": args.beams,
                       "vit": args.vit, "gpt2": args.gpt2, "batch_per_gpu": B, "global_batch": world * B,
                       "frames": T, "max_new_tokens": args.max_new,
                       "decode": args.decode if args.beams == 1 else f"beam-{args.beams} (device beam search, HF _beam_search)",
                       "vit_precision": args.precision, "decoder_precision": args.dec_precision,
                       "lm_head": ("bf16 screen + exact f32 rescoring" if dec.screen and args.beams == 1
                                   and args.decode == "hf_greedy" or dec.screen and args.decode == "raw_greedy"
                                   else args.dec_precision),
                       "hipgraph_decode": not args.no_graph, "parallelism": f"dp{world}",
                       "decode_block_cap": cfg.max_blocks,
                       "schedule": "serial" if args.serial else
                       f"CU-masked encode stream (off {args.reserve_cus} CUs) overlapped with {args.dec_lanes} decode "
                       f"lane(s) in flight; each encode = {args.enc_group} consecutive batch(es) as one "
                       f"{args.enc_group * B}-video encode; each decode = {args.dec_group} consecutive batch(es) as one "
                       + (f"{args.dec_group * B}-row greedy decode graph" if args.beams == 1 else
                          f"{args.dec_group * B} x {args.beams}-beam search graph")
                       + (f"; decode lanes masked to {args.decode_cus} CUs (the {args.reserve_cus} the encode leaves "
                          f"free + {args.decode_cus - args.reserve_cus} of its)" if args.decode_cus > 0 and not args.serial
                          else ""),
                       "decode_cus": 0 if args.serial else args.decode_cus,
                       "dec_lanes": 1 if args.serial else args.dec_lanes,
                       "dec_group": 1 if args.serial else args.dec_group,
                       "enc_group": 1 if args.serial else args.enc_group},
            "value_definition": "pipelined throughput: videos captioned / wall time of the timed steps "
                                "(encodes overlapped with the decodes of earlier batches)",
            "captions_per_s_b_over_p50": world * B / (p50 / 1e3),
            # the reference's own throughput definition (batch / mean iteration wall time,
            # core/scripts/benchmark_baseline.py:291-292, 356-358) on the same per-batch latencies
            "captions_per_s_b_over_mean": world * B / (statistics.mean(lat) / 1e3),
            "p50_latency_ms": p50,
            "new_tokens_per_caption": {"mean": sum(lens) / len(lens), "max": max(lens),
                                       "decode_steps_run": args.max_new},
            "stage_ms_p50": {"vit_encode_prefix": statistics.median(vit_ms),
                             "prefix_ready_to_ids": statistics.median(dec_ms)},
            # the reference's per-stage statistics (core/scripts/benchmark_baseline.py:114-139) over the
            # timed steps: batch latency (encode start -> ids), encode (+ prefix), prefix-ready -> ids
            "latency_ms_stats": {"end_to_end": describe(lat), "vit_encode_prefix": describe(vit_ms),
                                 "prefix_ready_to_ids": describe(dec_ms)},
            "roofline": {"bound": "mfma",
                         "kernel": {"bf16": "vit.fc1 vcap_gemm256_kernel<bf16,bf16,1>",
                                    "fp8": "vit.fc1 vcap_gemm256_kernel<mxfp8,mxfp8,4>"}.get(
                                        args.precision, "vit.fc1 vcap_gemm256_kernel<f32,f32,1>"),
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                         "traffic": fc1_traffic(M, va.mlp, va.dim) if args.precision == "bf16" else None,
                         "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "flops_per_launch": fc1["flops_per_launch"], "avg_launch_ms": fc1["avg_launch_ms"],
                         "launch_rows": M, "launches": fc1["launches"],
                         "timing": "HIP events around each fc1 launch on its stream inside the timed region "
                                   "(vcap_probe_*), read right after it; priced per launch population",
                         "other_populations": fc1["other_populations"]},
            "attention": {"kernel": ("vit.attention = vcap_vit_qkv_attention kernel (QKV projection + attention)"
                                     if fused_attn else "vit.attention"),
                          "bound": "mfma" if fused_attn else "hbm", "avg_launch_ms": att["avg_launch_ms"],
                          "launch_rows": M, "launches": att["launches"],
                          "achieved_tflops": att["flops_per_launch"] / (att["avg_launch_ms"] / 1e3) / 1e12,
                          "frac_of_mfma_peak": att["flops_per_launch"] / (att["avg_launch_ms"] / 1e3) / 1e12 / peak,
                          "bytes_per_launch": att["bytes_per_launch"],
                          "achieved_gbs": att["bytes_per_launch"] / (att["avg_launch_ms"] / 1e3) / 1e9,
                          "frac_of_hbm_peak": att["bytes_per_launch"] / (att["avg_launch_ms"] / 1e3) / 1e9 / PEAK_HBM_GBS,
                          "other_populations": att["other_populations"]},
            # whole-path roofline: executed ViT FLOPs at the MFMA peak + the decode's
            # weight bytes (every token step streams all projection weights + the tied lm_head) at
            # the HBM peak, against the measured time per batch
            "path_roofline": {"t_roof_ms": t_roof * 1e3, "t_measured_ms": elapsed / args.steps * 1e3,
                              "frac": t_roof / (elapsed / args.steps),
                              "vit_tflop": vit_exec / 1e12, "decode_weight_gb": dec_bytes / 1e9},
            "strict_batch": strict,
            "token_exact": None,
            "batch_sweep": sweep,
            "pmc": pmc_summary(args.vit, args.gpt2, M, args.precision),
            "parity": parity,
            "decode_roofline": dec_alone,
            "vit_flops_per_step": B * T * va.flops_per_frame(),
            "vit_flops_per_step_executed": B * T * va.flops_per_frame(cls_tail=True),
            "launch": {"launcher": launcher_name(), "world_size": world, "visible_gpus": torch.cuda.device_count(),
                       "backend": backend if world > 1 else None,
                       "gpu_per_rank": "LOCAL_RANK % visible GPUs (one process per GPU)"},
        }
        if host_lat:
            hp50 = statistics.median(host_lat)
            out["host_e2e"] = {"p50_ms": hp50 * 1e3, "captions_per_s": world * B / hp50, "iters": len(host_lat),
                               "stats_ms": describe([x * 1e3 for x in host_lat]),
                               "h2d_bytes": int(video.numel() * video.element_size()),
                               "what": "pinned host fp32 frames -> H2D -> encode -> decode -> ids on host, "
                                       "one batch at a time (no overlap; rank 0's clock)"}
        if world == 1 and args.cpu_baseline_s > 0:
            cb = cpu_baseline(sd, va, ga, frames_np, args.cpu_baseline_s, args.max_new, args.beams)
            ref_ids = cb.pop("_ids")
            out["cpu_baseline"] = cb
            out["oracle_parity"] = oracle_agreement(last, ref_ids, ga.eos_token_id, args.beams)
            if args.precision == "fp32" and args.dec_precision == "fp32":
                out["parity"] = out["oracle_parity"]
            if token_exact is not None:
                token_exact["oracle_parity"] = oracle_agreement(token_exact["_last"], ref_ids, ga.eos_token_id)
        else:
            out["cpu_baseline"] = None
        if token_exact is not None:
            token_exact.pop("_last", None)
            out["token_exact"] = token_exact
        if args.export_csv or args.export_json:
            export(args, out, B, lat, vit_ms, dec_ms, ids_all, dec_alone, sweep_rows, ga.eos_token_id,
                   torch.cuda.max_memory_allocated(dev) / 2**20)
        print(json.dumps(out), flush=True)
    pipe.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
