"""Per-phase timeline of the persistent decode (diagnostic build switch VCAP_PERSIST_FLAGS=8: the sync
wave stamps s_memrealtime, 100 MHz, at each phase's barrier arrival and release).  For each phase kind
(P1 ln_1 + c_attn, P2 attention, P3 attn c_proj, P4 ln_2 + c_fc, P5 mlp c_proj, P6 lm_head, P7
finalize): the work span (previous release -> this arrival; mean over workgroups and the slowest
workgroup), and the barrier span (last arrival -> release, mean over workgroups).
usage: VCAP_PERSIST_FLAGS=8 python tools/persist_stamps.py [B] [G]"""
import ctypes as C
import os
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
    assert int(os.environ.get("VCAP_PERSIST_FLAGS", "0")) & 8, "set VCAP_PERSIST_FLAGS=8"
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 96
    dev = torch.device("cuda:0")
    ga = configs.gpt2_arch("gpt2")
    sd = weights.synthetic_state_dict(1, configs.vit_arch("vit_tiny_test"), ga)
    dec = HipGPT2Decoder(sd, ga, "bf16", dev)
    prefix = torch.from_numpy((np.random.default_rng(B).standard_normal((B, 4, ga.n_embd)) * 0.5)
                              .astype(np.float32)).to(dev)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True, persistent=G)
    for _ in range(3):
        dec.generate_ids(prefix, [ga.bos_token_id], cfg)
    torch.cuda.synchronize()
    L = ga.n_layer
    per_step = 5 * L + 2
    nph = 23 * per_step
    n = 256 * 2048 * 2
    buf = (C.c_ulong * n)()
    assert N.lib().vcap_persist_stamps_read(buf, C.c_size_t(n)) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 2048, 2)[:G, :nph].astype(np.int64)
    arr, rel = st[:, :, 0], st[:, :, 1]
    prev_rel = np.concatenate([arr[:, :1], rel[:, :-1]], axis=1)   # phase 0: from its own arrival
    work = (arr - prev_rel) * 10.0 / 1e3                  # ns -> us (100 MHz ticks = 10 ns)
    last_arr = arr.max(axis=0)
    bar = (rel - last_arr[None, :]) * 10.0 / 1e3
    span = (rel.max(axis=0) - np.concatenate([[arr.min()], rel.max(axis=0)[:-1]])) * 10.0 / 1e3
    kinds = ["P1 ln_1+c_attn", "P2 attention", "P3 attn c_proj", "P4 ln_2+c_fc", "P5 mlp c_proj"]
    label = [kinds[i % 5] if i < 5 * L else ("P6 lm_head" if i == 5 * L else "P7 finalize") for i in range(per_step)]
    print(f"B={B} G={G}: {nph} phases, total {float((rel.max() - arr.min()) * 10 / 1e3):.1f} us "
          f"({float((rel.max() - arr.min()) * 10 / 1e3 / 23):.1f} us per step)")
    print(f"{'phase':16s} {'work mean':>10s} {'work max':>10s} {'barrier':>9s} {'phase span':>11s}  (us, per phase)")
    for k in dict.fromkeys(label):
        idx = [i for i in range(nph) if label[i % per_step] == k and i >= per_step]  # skip the first step
        w = work[:, idx]
        print(f"{k:16s} {w.mean():10.2f} {w.max(axis=0).mean():10.2f} {bar[:, idx].mean():9.2f} "
              f"{span[idx].mean():11.2f}")


if __name__ == "__main__":
    main()
