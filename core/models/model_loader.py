"""Backend switch (reference core/models/model_loader.py:13-28) with the MI355X HIP backend.

`load_caption_model(config)` keeps the reference's error semantics: "tensorrt" (or
config.tensorrt.enabled) -> NotImplementedError, any other unknown backend -> ValueError.  The
reference's "torch" eager backend is not part of this framework (no CPU/eager fallback exists);
asking for it raises ValueError naming the supported backend.
"""
from __future__ import annotations

import logging

from core.config import InferenceConfig

log = logging.getLogger(__name__)
SUPPORTED_BACKENDS = ("hip",)


def load_caption_model(config: InferenceConfig):
    backend = (config.backend or "").lower()
    if config.tensorrt.enabled or backend == "tensorrt":
        raise NotImplementedError("TensorRT backend hook is reserved but not implemented (use backend='hip').")
    if backend not in SUPPORTED_BACKENDS:
        raise ValueError(f"Unsupported inference backend: {config.backend} (supported: {SUPPORTED_BACKENDS})")
    return load_hip_caption_model(config)


def load_hip_caption_model(config: InferenceConfig):
    from vcap.caption import HipVideoCaptionModel, build_state_dict
    sd = build_state_dict(config.ckpt, config.vit_name, config.gpt2_name, config.weights_seed, config.prefix_len)
    model = HipVideoCaptionModel(sd, config.vit_name, config.gpt2_name, config.prefix_len, config.precision,
                                 config.device, config.tokenizer_dir, config.use_hipgraph,
                                 decoder_precision=config.decoder_precision)
    log.info("loaded %s (%s) + %s (%s decoder) on %s", config.vit_name, config.precision, config.gpt2_name,
             model.decoder_precision, config.device)
    return model
