"""Instruction counts of the bench's ViT attention kernel (vcap_vit_attention_bf16_kernel<14,13,8,false>,
ViT-B/16: 197 tokens -> 13 query tiles and 14 key tiles of 16) from its gfx950 assembly, and the issue- and
traffic-bound ceilings on its MFMA utilisation that follow.  Runs on the CPU (hipcc -S).

usage: python tools/attn_isa_counts.py [kernel-suffix]   (default ILi14ELi13ELi8ELb0E)"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "video-caption-algorithm_amd" / "csrc"
suffix = sys.argv[1] if len(sys.argv) > 1 else "ILi14ELi13ELi8ELb0E"

with tempfile.TemporaryDirectory() as td:
    asm = Path(td) / "attn.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-honor-nans",
                    f"-I{CSRC}", f"-I{ROOT / 'include'}", "--cuda-device-only", "-S",
                    str(CSRC / "vit_attention.hip"), "-o", str(asm)], check=True, capture_output=True)
    lines = asm.read_text().split("\n")

st = next(i for i, l in enumerate(lines) if l.startswith("_Z30vcap_vit_attention_bf16_kernel" + suffix)
          and l.split(";")[0].strip().endswith(":"))
name = lines[st].split(":")[0]
en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith("s_endpgm"))
body = lines[st:en + 1]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}


def cls(op):
    if op.startswith("v_mfma"):
        return op
    if op.startswith("v_exp"):
        return "v_exp (transcendental)"
    if op.startswith("v_permlane"):
        return "v_permlane*_swap"
    if op.startswith("v_"):
        return "other VALU"
    if op.startswith("ds_read_b64_tr"):
        return "ds_read_b64_tr_b16"
    if op.startswith("ds_"):
        return "other LDS"
    if op.startswith(("global_", "buffer_")):
        return "VMEM (incl. LDS-DMA)"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    return "SALU / branch"


# the query-tile bodies: the straight-line regions between the kernel's two forward branches to the
# epilogue exit (a wave runs one or two 16-query tiles; its key loop is fully unrolled)
branches = []
for i, l in enumerate(body):
    m = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m:
        branches.append((i, labels[m.group(1)]))
exit_line = max(t for _, t in branches)
cuts = sorted({i for i, t in branches if t == exit_line})
regions = [("whole kernel", 0, len(body))]
if len(cuts) >= 2:
    regions += [("query tile 1", cuts[0], cuts[1]), ("query tile 2 (waves 0-4)", cuts[1], cuts[-1])]


def count(a, b):
    c = collections.Counter()
    for l in body[a:b]:
        t = l.strip()
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            c[cls(t.split()[0])] += 1
    return c


print(f"kernel {name}")
print(f"{len(body)} assembly lines; branches: " + ", ".join(f"{i}->{t}{' (back)' if t < i else ''}" for i, t in branches))
tile = None
for title, a, b in regions:
    c = count(a, b)
    print(f"\n[{title}] lines {a}-{b}")
    for k, v in sorted(c.items(), key=lambda x: -x[1]):
        print(f"  {v:5d}  {k}")
    if title == "query tile 1":
        tile = c

tiles = {t: count(a, b) for t, a, b in regions[1:]}
flop = 4 * 256 * 12 * 197 * 197 * 64        # one 16-video launch: 256 frames x 12 heads
byts = 256 * 197 * (3 * 768 + 768) * 2     # q, k, v in + out, bf16
useful = (197 / 208) * (197 / 224)         # 197 of 208 queries x 197 of 224 padded keys
print("\nissue model per 16-query tile and wave (MI355X_MICROARCH.md 'vector-instruction ISSUE cost'): a 16x16x32 "
      "bf16 MFMA takes the matrix pipe 16 cycles and holds the SIMD's vector issue 8 of them, v_exp 8, other VALU "
      "4; LDS reads issue on their own port")
for t, c in tiles.items():
    mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
    valu = c["other VALU"] + c["v_permlane*_swap"]
    ex = c["v_exp (transcendental)"]
    pipe, issue = mf * 16, valu * 4 + ex * 8 + mf * 8
    frac = pipe / max(pipe, issue)
    print(f"  {t}: {mf} MFMA = {pipe} pipe cycles; {valu} VALU + {ex} v_exp + {mf} x 8 MFMA hold = {issue} issue "
          f"cycles -> matrix pipe busy <= {frac:.2f}; x {useful:.2f} useful -> <= {frac * useful:.2f} of the dense "
          "peak (algorithmic), with both waves of a SIMD perfectly interleaved")
print(f"\ntraffic: {byts / 1e6:.0f} MB per 16-video launch (q, k, v read once + output), {flop / 1e9:.1f} GFLOP")
for bw in (8.0, 6.3):
    t = byts / (bw * 1e12)
    print(f"  at {bw} TB/s: {t * 1e6:.1f} us -> MFMA utilisation <= {flop / t / 2.5e15:.2f} of the 2.5 PF/s bf16 dense peak")
