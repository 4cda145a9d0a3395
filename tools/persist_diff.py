"""Where the persistent decode's logits first differ from the launch chain's (diagnostic).
usage: python tools/persist_diff.py [B] [G] [raw]"""
import dataclasses
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402
from vcap import configs, weights  # noqa: E402
from vcap.model import GenConfig, HipGPT2Decoder  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    raw = len(sys.argv) > 3 and sys.argv[3] == "raw"
    dev = torch.device("cuda:0")
    ga = configs.gpt2_arch("gpt2")
    sd = weights.synthetic_state_dict(1, configs.vit_arch("vit_tiny_test"), ga)
    dec = HipGPT2Decoder(sd, ga, "bf16", dev)
    prefix = torch.from_numpy((np.random.default_rng(B + G).standard_normal((B, 4, ga.n_embd)) * 0.5)
                              .astype(np.float32)).to(dev)
    cfg = GenConfig.raw_greedy(24, ga.eos_token_id) if raw else GenConfig(24, 8, 3, 1.1, ga.eos_token_id,
                                                                             ga.eos_token_id, True)
    runs = []
    for g in (0, 0, G, G, 0):
        lg = torch.full((24, B, ga.vocab), float("nan"), device=dev)
        ids = dec.generate_ids(prefix, [ga.bos_token_id], dataclasses.replace(cfg, persistent=g), logits_out=lg)
        torch.cuda.synchronize()
        runs.append((g, ids.cpu().numpy(), lg.cpu()))
    for a in range(len(runs)):
        for b in range(a + 1, len(runs)):
            d = float((runs[a][2] - runs[b][2]).abs().max())
            print(f"run {a} (G={runs[a][0]}) vs run {b} (G={runs[b][0]}): max |d logits| {d:.3e}, "
                  f"ids equal {np.array_equal(runs[a][1], runs[b][1])}")
    (_, i0, l0), (_, i1, l1) = runs[0], runs[2]
    print("faults", N.lib().vcap_decode_faults(), "ids equal", np.array_equal(i0, i1))
    for s in range(24):
        d = (l0[s] - l1[s]).abs()
        nd = int((d > 0).sum())
        if nd:
            rows = sorted(set(int(r) for r in (d > 0).nonzero()[:, 0]))
            print(f"step {s}: {nd} logits differ, max |d| {float(d.max()):.3e}, rows {rows}, "
                  f"ids equal at this step {np.array_equal(i0[:, s], i1[:, s])}")
        else:
            print(f"step {s}: identical")


if __name__ == "__main__":
    main()
