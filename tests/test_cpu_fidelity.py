"""Host logic of the fidelity evidence (vcap/fidelity.py) and the bench's per-launch roofline
pricing (bench.launch_summary / describe), on synthetic data - no GPU."""
import importlib.util
from pathlib import Path

import numpy as np
import torch

from vcap import fidelity
from vcap.model import GenConfig

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _greedy(logits, cfg):
    """Reference greedy ids from raw logits [L, B, V] along their own argmax path."""
    from vcap.search import _processors
    L, B, _ = logits.shape
    ids = torch.zeros(B, L, dtype=torch.long)
    for s in range(L):
        sc = _processors(logits[s].double(), ids[:, :s], cfg.repetition_penalty, cfg.no_repeat_ngram_size,
                         cfg.min_new_tokens, cfg.eos_token_id)
        ids[:, s] = sc.argmax(-1)
    return ids


def test_greedy_divergence_explains_a_near_tie():
    g = torch.Generator().manual_seed(0)
    L, B, V = 6, 3, 40
    cfg = GenConfig(L, 0, 0, 1.0, V - 1, V - 1, False)   # raw greedy: processors off
    ref = torch.randn(L, B, V, generator=g) * 3
    ref[:, :, V - 1] = -50.0                              # no EOS
    ids = _greedy(ref, cfg)
    # caption 1: a near-tie at step 2 between its token and another one
    a = int(ids[1, 2])
    other = (a + 1) % (V - 1)
    ref[2, 1, other] = ref[2, 1, a] - 0.004
    ids = _greedy(ref, cfg)
    test_tf = ref + 0.01 * torch.randn(L, B, V, generator=g).clamp(-1, 1)
    test_tf[2, 1, a] = ref[2, 1, a]
    test_tf[2, 1, other] = ref[2, 1, a] + 0.001           # the tested precision prefers `other`
    test_ids = ids.clone()
    test_ids[1, 2:] = torch.tensor([other] + [0] * (L - 3))
    rep = fidelity.greedy_divergence(test_ids.numpy(), ids.numpy(), ref, test_tf, cfg)
    assert rep["captions_identical"] == 2 and len(rep["divergences"]) == 1
    d = rep["divergences"][0]
    assert (d["caption"], d["step"], d["ref_token"], d["test_token"]) == (1, 2, a, other)
    assert abs(d["fp32_margin"] - 0.004) < 1e-5 and d["test_prefers_its_token"]
    assert rep["every_divergence_within_error"] and rep["lead_at_least_guaranteed"]
    assert rep["max_raw_logit_err"] <= 0.0141


def test_bench_launch_summary_prices_each_population():
    b = _bench()
    launches = [(0.30, 50432)] * 10 + [(0.16, 25216)] * 2
    s = b.launch_summary(launches, 50432, lambda r: 2.0 * r * 3072 * 768, lambda r: float(r))
    assert s["launches"] == 10 and abs(s["avg_launch_ms"] - 0.30) < 1e-12
    assert s["flops_per_launch"] == 2.0 * 50432 * 3072 * 768 and s["bytes_per_launch"] == 50432.0
    assert s["other_populations"] == {"25216": {"launches": 2, "avg_launch_ms": 0.16}}
    st = b.describe([1.0, 2.0, 3.0, 4.0])
    assert st["mean"] == 2.5 and st["min"] == 1.0 and st["max"] == 4.0 and st["n"] == 4
    assert abs(st["std"] - np.std([1, 2, 3, 4])) < 1e-12 and 3.9 < st["p99"] <= 4.0
