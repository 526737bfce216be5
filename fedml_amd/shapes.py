"""State-dict key/shape/dtype lists of the BASELINE.json configurations.

Used to build synthetic client updates of the exact structure the reference
aggregates; no weights or datasets are needed.  Each entry is
``(key, shape, dtype)`` in the model's state_dict order.

- ``lr_mnist``      python/fedml/model/linear/lr.py:4 (784 -> 10), config 1
- ``cnn_web``       python/fedml/model/cv/cnn.py:169-186, 62,006 params, config 2
- ``resnet50``      torchvision ResNet-50 (Bottleneck [3,4,6,3]), config 3:
                    25,557,032 params, 25,610,152 float elements, 53 int64
- ``vit_b16``       torchvision ViT-B/16, 152 entries, 86,567,656 elements, config 4
- ``llama2_7b_lora`` PEFT LoRA r=8 on q_proj/v_proj of Llama-2-7B, config 5
"""
from __future__ import annotations

from typing import List, Tuple

import torch

Entry = Tuple[str, Tuple[int, ...], torch.dtype]


def _bn(prefix: str, c: int) -> List[Entry]:
    return [
        (f"{prefix}.weight", (c,), torch.float32),
        (f"{prefix}.bias", (c,), torch.float32),
        (f"{prefix}.running_mean", (c,), torch.float32),
        (f"{prefix}.running_var", (c,), torch.float32),
        (f"{prefix}.num_batches_tracked", (), torch.int64),
    ]


def lr_mnist(in_dim: int = 784, out_dim: int = 10) -> List[Entry]:
    return [("linear.weight", (out_dim, in_dim), torch.float32), ("linear.bias", (out_dim,), torch.float32)]


def cnn_web() -> List[Entry]:
    f = torch.float32
    return [
        ("conv1.weight", (6, 3, 5, 5), f), ("conv1.bias", (6,), f),
        ("conv2.weight", (16, 6, 5, 5), f), ("conv2.bias", (16,), f),
        ("fc1.weight", (120, 400), f), ("fc1.bias", (120,), f),
        ("fc2.weight", (84, 120), f), ("fc2.bias", (84,), f),
        ("fc3.weight", (10, 84), f), ("fc3.bias", (10,), f),
    ]


def resnet50(num_classes: int = 1000) -> List[Entry]:
    f = torch.float32
    out: List[Entry] = [("conv1.weight", (64, 3, 7, 7), f)] + _bn("bn1", 64)
    inplanes = 64
    for li, (planes, blocks) in enumerate(zip((64, 128, 256, 512), (3, 4, 6, 3)), start=1):
        for b in range(blocks):
            p = f"layer{li}.{b}"
            out.append((f"{p}.conv1.weight", (planes, inplanes, 1, 1), f))
            out += _bn(f"{p}.bn1", planes)
            out.append((f"{p}.conv2.weight", (planes, planes, 3, 3), f))
            out += _bn(f"{p}.bn2", planes)
            out.append((f"{p}.conv3.weight", (planes * 4, planes, 1, 1), f))
            out += _bn(f"{p}.bn3", planes * 4)
            if b == 0:
                out.append((f"{p}.downsample.0.weight", (planes * 4, inplanes, 1, 1), f))
                out += _bn(f"{p}.downsample.1", planes * 4)
            inplanes = planes * 4
    out += [("fc.weight", (num_classes, 2048), f), ("fc.bias", (num_classes,), f)]
    return out


def vit_b16(dtype: torch.dtype = torch.bfloat16, num_classes: int = 1000) -> List[Entry]:
    d, mlp, L = 768, 3072, 12
    out: List[Entry] = [
        ("class_token", (1, 1, d), dtype),
        ("conv_proj.weight", (d, 3, 16, 16), dtype),
        ("conv_proj.bias", (d,), dtype),
        ("encoder.pos_embedding", (1, 197, d), dtype),
    ]
    for i in range(L):
        p = f"encoder.layers.encoder_layer_{i}"
        out += [
            (f"{p}.ln_1.weight", (d,), dtype), (f"{p}.ln_1.bias", (d,), dtype),
            (f"{p}.self_attention.in_proj_weight", (3 * d, d), dtype),
            (f"{p}.self_attention.in_proj_bias", (3 * d,), dtype),
            (f"{p}.self_attention.out_proj.weight", (d, d), dtype),
            (f"{p}.self_attention.out_proj.bias", (d,), dtype),
            (f"{p}.ln_2.weight", (d,), dtype), (f"{p}.ln_2.bias", (d,), dtype),
            (f"{p}.mlp.0.weight", (mlp, d), dtype), (f"{p}.mlp.0.bias", (mlp,), dtype),
            (f"{p}.mlp.3.weight", (d, mlp), dtype), (f"{p}.mlp.3.bias", (d,), dtype),
        ]
    out += [
        ("encoder.ln.weight", (d,), dtype), ("encoder.ln.bias", (d,), dtype),
        ("heads.head.weight", (num_classes, d), dtype), ("heads.head.bias", (num_classes,), dtype),
    ]
    return out


def llama2_7b_lora(r: int = 8, hidden: int = 4096, layers: int = 32) -> List[Entry]:
    f = torch.float32
    out: List[Entry] = []
    for i in range(layers):
        for proj in ("q_proj", "v_proj"):
            p = f"base_model.model.model.layers.{i}.self_attn.{proj}"
            out += [(f"{p}.lora_A.weight", (r, hidden), f), (f"{p}.lora_B.weight", (hidden, r), f)]
    return out


MODELS = {
    "lr_mnist": lr_mnist,
    "cnn_web": cnn_web,
    "resnet50": resnet50,
    "vit_b16": vit_b16,
    "llama2_7b_lora": llama2_7b_lora,
}


_BUFFER_SUFFIXES = (".running_mean", ".running_var", ".num_batches_tracked")


def param_names(entries: List[Entry]) -> List[str]:
    """The named parameters of these state-dict entries (model.named_parameters()
    order): everything but BatchNorm's registered buffers.  What FedOpt steps
    (FedOptAggregator.py:118-125); buffers take the average."""
    return [k for k, _, _ in entries if not k.endswith(_BUFFER_SUFFIXES)]


def numel(entries: List[Entry], dtype: torch.dtype | None = None) -> int:
    tot = 0
    for _, shape, dt in entries:
        if dtype is None or dt == dtype:
            n = 1
            for s in shape:
                n *= s
            tot += n
    return tot
