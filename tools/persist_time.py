"""Decode step time alone on the GPU: the launch chain (persistent=0) against the persistent decode
at several grid sizes.  step = (t[24-token graph] - t[2-token graph]) / 22, both replayed after
warm-up (the prefill and step 0 cancel).  usage: python tools/persist_time.py [B ...]"""
import dataclasses
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402
from vcap import configs, weights  # noqa: E402
from vcap.model import GenConfig, HipGPT2Decoder  # noqa: E402


def replay_s(dec, prefix, cfg, ga, reps=30):
    out = torch.empty(prefix.shape[0], cfg.max_new_tokens, dtype=torch.int32, device=prefix.device)
    for _ in range(3):
        dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, out.cpu()


def main():
    gpt2 = "gpt2"
    Bs = [int(x) for x in sys.argv[1:]] or [8, 16]
    dev = torch.device("cuda:0")
    ga = configs.gpt2_arch(gpt2)
    sd = weights.synthetic_state_dict(1, configs.vit_arch("vit_tiny_test"), ga)
    dec = HipGPT2Decoder(sd, ga, "bf16", dev)
    for B in Bs:
        prefix = torch.from_numpy((np.random.default_rng(B).standard_normal((B, 4, ga.n_embd)) * 0.5)
                                  .astype(np.float32)).to(dev)
        base = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
        ref = None
        gs = os.environ.get("PERSIST_GS")
        for G in ([int(x) for x in gs.split(",")] if gs else (0, 96, 128, 160, 192, 256)):
            t24, ids = replay_s(dec, prefix, dataclasses.replace(base, persistent=G), ga)
            t2, _ = replay_s(dec, prefix, dataclasses.replace(base, max_new_tokens=2, persistent=G), ga)
            ref = ids if ref is None else ref
            same = bool(torch.equal(ids, ref))
            print(f"B={B:2d} G={G:3d}: step {(t24 - t2) / 22 * 1e6:7.1f} us  24-token graph {t24 * 1e3:6.3f} ms  "
                  f"ids==chain {same}  faults {N.lib().vcap_decode_faults()}", flush=True)


if __name__ == "__main__":
    main()
