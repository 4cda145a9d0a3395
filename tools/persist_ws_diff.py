"""Which buffer, layer and cache position first differ between the launch chain and the persistent
decode (diagnostic).  Runs max_new = S tokens both ways on a zeroed private workspace and compares
the KV cache per (layer, position, row) and the final h / q / attn / act rows.
usage: python tools/persist_ws_diff.py [B] [G] [S]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vcap import configs, weights  # noqa: E402
from vcap.model import GenConfig, HipGPT2Decoder, _Workspace  # noqa: E402


def al(x):
    return (x + 255) & ~255


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    ga = configs.gpt2_arch("gpt2")
    sd = weights.synthetic_state_dict(1, configs.vit_arch("vit_tiny_test"), ga)
    dec = HipGPT2Decoder(sd, ga, "bf16", dev)
    prefix = torch.from_numpy((np.random.default_rng(B + G).standard_normal((B, 4, ga.n_embd)) * 0.5)
                              .astype(np.float32)).to(dev)
    E, L, H, V = ga.n_embd, ga.n_layer, ga.n_head, ga.vocab
    S0 = 4 + 1
    bufs = {}
    for g in (0, G):
        ws = _Workspace(dev)
        ws.get(dec.workspace_bytes(B, 1, S)).zero_()
        cfg = GenConfig(S, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, False, persistent=g)
        lg = torch.full((S, B, V), float("nan"), device=dev)
        ids = dec.generate_ids(prefix, [ga.bos_token_id], cfg, logits_out=lg, workspace=ws)
        torch.cuda.synchronize()
        bufs[g] = (ws.buf.cpu().numpy().copy(), ids.cpu().numpy(), lg.cpu().numpy())
    Mmax = B * S0
    maxp = (S0 + S + 15) // 16
    per_layer = B * maxp * H * 16 * 64
    off = {}
    o = 0
    for name, n in (("h", Mmax * E * 4), ("q", Mmax * E * 2), ("attn", Mmax * E * 2), ("act", Mmax * 4 * E * 2),
                    ("kc", per_layer * L * 2), ("vc", per_layer * L * 2)):
        off[name] = (o, n)
        o += al(n)
    (w0, i0, l0), (w1, i1, l1) = bufs[0], bufs[G]
    print(f"B={B} G={G} S={S}: ids equal {np.array_equal(i0, i1)}")
    for s in range(S):
        d = np.abs(l0[s] - l1[s])
        rows = sorted(set(np.nonzero(d > 0)[0].tolist()))
        print(f"step {s}: logits max |d| {float(np.nanmax(d)):.3e} rows {rows}")
    for name in ("kc", "vc"):
        o, n = off[name]
        a = w0[o:o + n].view(np.uint16).reshape(L, B, maxp, H, 16, 64)
        b = w1[o:o + n].view(np.uint16).reshape(L, B, maxp, H, 16, 64)
        diff = a != b
        print(f"{name}: {int(diff.sum())} elements differ")
        for ly in range(L):
            for pos in range(S0 + S - 1):
                dd = diff[ly, :, pos >> 4, :, pos & 15, :]
                if dd.any():
                    r, h, dch = np.nonzero(dd)
                    fa = (a[ly, :, pos >> 4, :, pos & 15, :].astype(np.uint32) << 16).view(np.float32)
                    fb = (b[ly, :, pos >> 4, :, pos & 15, :].astype(np.uint32) << 16).view(np.float32)
                    print(f"  {name} layer {ly} pos {pos}: rows {sorted(set(r.tolist()))} heads "
                          f"{sorted(set(h.tolist()))[:12]} n {len(r)} max |d| {float(np.abs(fa - fb).max()):.3e}")
    for name, dt, width in (("h", np.float32, E), ("q", np.uint16, E), ("attn", np.uint16, E), ("act", np.uint16, 4 * E)):
        o, n = off[name]
        a = w0[o:o + n].view(dt).reshape(-1, width)[:B]
        b = w1[o:o + n].view(dt).reshape(-1, width)[:B]
        rows = sorted(set(np.nonzero(a != b)[0].tolist()))
        print(f"{name}: rows differing {rows}")


if __name__ == "__main__":
    main()
