#!/usr/bin/env python3
"""Per-stage kernel time under rocprofv3, the reference's profile harness restated
(core/scripts/benchmark_baseline.py:265-286 `run_one_iteration`, :160-240 `run_decoder_steps`;
core/scripts/profile_nsight.py:24-34): each iteration runs ViT_Encoder (the encoder), then
Cross_Modal_Alignment (proj + engine LN-scale + mapper), then GPT2_Decoder_Step (the reference's
raw per-token loop through `decoder.model(inputs_embeds=, past_key_values=)`, one
GPT2_Decoder_Step/token_NN range per token), each stage synchronised as the reference's
`cuda_stage` does, inside roctx ranges (vcap/trace.py).  Then `--pipeline-steps` batches of the
bench's pipelined schedule with the pipeline's own ranges (ViT_Encoder around each fused encode
launch, GPT2_Decoder_Step around each decode-graph launch; run it as its own profile, `--iters 0`,
as it uses the same range names).

    cd /tmp && rocprofv3 --marker-trace --kernel-trace --kernel-rename --stats -d OUT -o run -- \\
        python3 /root/repo/tools/stage_profile.py
    python3 tools/stage_profile.py --summarize OUT      # -> per-stage table (JSON + text)

`--kernel-rename` names each kernel after the innermost range it was dispatched in, so the kernel
statistics group by stage.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
sys.path.insert(0, str(ROOT))


def run(args):
    import torch
    from vcap import configs, prng, trace, weights
    from vcap.caption import HipGPT2LMHead, _WTE
    from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder
    from vcap.pipeline import CaptionPipeline

    trace.enable()
    dev = torch.device("cuda", 0)
    va, ga = configs.vit_arch(args.vit), configs.gpt2_arch(args.gpt2)
    sd = weights.synthetic_state_dict(1, va, ga)
    video = torch.from_numpy(prng.imagenet_frames(1000, (args.batch, args.frames, 3, va.image, va.image))).to(dev)
    enc = HipViTEncoder(sd, va, args.precision, dev)
    pre = HipPrefix(sd, ga.n_embd, device=dev)
    dec = HipGPT2Decoder(sd, ga, args.dec_precision, dev)
    lm = HipGPT2LMHead(dec, ga, _WTE(dec.wte, sd["decoder.model.transformer.wte.weight"]))
    bos = torch.full((args.batch, 1), ga.bos_token_id, dtype=torch.long, device=dev)
    stage_ms = defaultdict(list)

    def stage(name, fn):
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        with trace.range(name):
            start.record()
            out = fn()
            end.record()
            torch.cuda.synchronize(dev)
        stage_ms[name].append(start.elapsed_time(end))
        return out

    def decoder_steps(prefix):
        x = torch.cat([prefix, lm.transformer.wte(bos)], dim=1)
        past, done = None, torch.zeros(args.batch, dtype=torch.bool, device=dev)
        for i in range(args.max_new):
            with trace.range(f"{trace.DECODE}/token_{i:02d}"):
                out = lm(inputs_embeds=x, past_key_values=past, use_cache=True)
                torch.cuda.synchronize(dev)
            tok = out.logits[:, -1, :].argmax(-1)
            tok = torch.where(done, torch.full_like(tok, ga.eos_token_id), tok)
            done |= tok == ga.eos_token_id
            past = out.past_key_values
            if bool(done.all()):
                break
            x = lm.transformer.wte(tok).unsqueeze(1)

    for it in range(args.iters + 1):           # iteration 0 = warm-up (ranges too: named "warmup/...")
        tag = "" if it else "warmup/"
        emb = stage(tag + trace.VIT, lambda: enc.encode(video, None)[0])
        pfx = stage(tag + trace.ALIGN, lambda: pre.project(emb))
        stage(tag + trace.DECODE, lambda: decoder_steps(pfx))
    if args.pipeline_steps > 0:
        cfg = GenConfig(args.max_new, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
        cfg.max_blocks = 96
        pipe = CaptionPipeline(enc, pre, dec, cfg, args.batch, [ga.bos_token_id], dev, reserve_cus=32, dec_lanes=2,
                               dec_group=2, enc_group=2)
        for _ in range(args.pipeline_steps):
            pipe.submit(video)
        pipe.synchronize()
        pipe.close()
    torch.cuda.synchronize(dev)
    summary = {k: {"n": len(v), "mean_ms": sum(v) / len(v)} for k, v in stage_ms.items() if not k.startswith("warmup/")}
    print(json.dumps({"stage_ms_host_events": summary}), flush=True)


def summarize(out_dir: str):
    """kernel_stats of a --kernel-rename run (kernel names = innermost roctx range) -> per-stage totals,
    plus the marker ranges' own wall time."""
    files = glob.glob(os.path.join(out_dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_stats.csv under {out_dir}")
    by_stage = defaultdict(lambda: {"calls": 0, "total_ns": 0.0, "names": set()})
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row["Name"]
                if name.startswith("warmup/"):
                    continue
                key = name.split("/token_")[0] if name.startswith(("GPT2_Decoder_Step", "ViT_Encoder",
                                                                 "Cross_Modal_Alignment")) else "(outside ranges)"
                d = by_stage[key]
                d["calls"] += int(row["Calls"])
                d["total_ns"] += float(row["TotalDurationNs"])
                d["names"].add(name)
    tot = sum(d["total_ns"] for d in by_stage.values())
    out = {k: {"kernel_calls": d["calls"], "kernel_ms": d["total_ns"] / 1e6,
               "share": d["total_ns"] / tot if tot else 0.0, "ranges": len(d["names"])}
           for k, d in sorted(by_stage.items(), key=lambda kv: -kv[1]["total_ns"])}
    print(json.dumps({"kernel_time_by_stage": out, "source": files}, indent=1))
    for k, d in out.items():
        print(f"{k:28s} {d['kernel_calls']:8d} kernels {d['kernel_ms']:10.3f} ms  {100 * d['share']:5.1f} %")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize", default="", help="rocprofv3 output directory to summarise (no GPU work)")
    ap.add_argument("--vit", default="vit_base_patch16_224")
    ap.add_argument("--gpt2", default="gpt2")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--dec-precision", default="fp32", help="the reference's decoder arithmetic by default")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--max-new", type=int, default=24)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--pipeline-steps", type=int, default=0,
                    help="> 0: (run separately, --iters 0) batches of the pipelined schedule with its own ranges")
    args = ap.parse_args()
    if args.summarize:
        summarize(args.summarize)
    else:
        run(args)


if __name__ == "__main__":
    main()
