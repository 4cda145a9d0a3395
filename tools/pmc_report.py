"""Summarise the tools/pmc.sh passes of `bench.py --serial` into profiles/<name>.json:
per-kernel FETCH/WRITE bytes (FETCH_SIZE doubled: gfx950 reports half of 16-B-per-lane streaming
reads, MI355X_MICROARCH.md), MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs), LDS bank conflicts; plus the decode's HBM bytes per token step.
usage: python tools/pmc_report.py <pmc outdir> <token steps in the run> <out.json> [ViT rows per launch]"""
import csv
import glob
import json
import sys
from collections import defaultdict

out_dir, token_steps, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vit_rows = int(sys.argv[4]) if len(sys.argv) > 4 else 25216
acc = defaultdict(lambda: defaultdict(list))
# attn-proj and fc2 run the same kernel (gemm256<bf16, f32, 2>, in-place f32 residual) on the same
# grid; in every pass they are dispatched alternately (per layer: attn-proj, then fc2), so their
# records are split by dispatch order into "...[attn-proj]" / "...[fc2]"
RESID = "vcap_gemm256_kernel<unsigned short, float, 2>"
for f in glob.glob(f"{out_dir}/*/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    resid_ids = sorted({int(r.get("Dispatch_Id", 0)) for r in rows if RESID in r.get("Kernel_Name", "")})
    role = {d: ("[attn-proj]" if i % 2 == 0 else "[fc2]") for i, d in enumerate(resid_ids)}
    for r in rows:
        name = r.get("Kernel_Name", "")
        if RESID in name:
            name = name.split("(")[0] + role[int(r.get("Dispatch_Id", 0))]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))


def avg(v):
    return sum(v) / len(v) if v else None


kernels = {}
dec_bytes = 0.0
for name, c in acc.items():
    short = (name if name.endswith("]") else name.split("(")[0]).replace("void ", "")
    fetch, write = avg(c.get("FETCH_SIZE", [])), avg(c.get("WRITE_SIZE", []))
    grbm, mfma = avg(c.get("GRBM_GUI_ACTIVE", [])), avg(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
    k = {"launches": len(c.get("GRBM_GUI_ACTIVE", [])),
         "fetch_bytes": fetch * 1000 * 2 if fetch is not None else None,
         "write_bytes": write * 1000 if write is not None else None,
         "mfma_util": mfma / (1024 * grbm / 8) if grbm and mfma is not None else None,
         "lds_bank_conflict_cycles": avg(c.get("SQ_LDS_BANK_CONFLICT", []))}
    kernels[short] = k
    if any(t in short for t in ("rows_gemv", "decode_attention", "decode_finalize")) and fetch is not None:
        dec_bytes += (sum(c["FETCH_SIZE"]) * 2 + sum(c.get("WRITE_SIZE", [0]))) * 1000
vit = {k: v for k, v in kernels.items()
       if "gemm256" in k or "vit_attention" in k or "qkv_attention" in k or "layernorm" in k}
res = {"source": "rocprofv3 --pmc passes (tools/pmc.sh) of python bench.py --serial --steps 2 --warmup 1",
       "vit_rows": vit_rows,
       "vit_kernels": vit,
       "decode": {"token_steps": token_steps, "hbm_bytes_per_token_step": dec_bytes / token_steps,
                  "algorithmic_weight_bytes_per_token_step": 247.1e6,
                  "note": "rows_gemv + decode attention + finalize kernels, FETCH x2 + WRITE; includes L2 misses "
                          "served by the Infinity Cache"},
       "all_kernels": kernels}
json.dump(res, open(dst, "w"), indent=1)
for k, v in vit.items():
    print(f"{k[:60]:60s} n={v['launches']:4d} fetch={v['fetch_bytes'] / 1e6 if v['fetch_bytes'] else 0:8.1f}MB "
          f"write={v['write_bytes'] / 1e6 if v['write_bytes'] else 0:8.1f}MB mfma={v['mfma_util'] or 0:.3f}")
print("decode bytes/token step", dec_bytes / token_steps / 1e6, "MB")
