"""UNet topology and state-dict layout of the reference's 9-channel inpainting UNet.

Mirrors the module construction order of code/unet.py:43-152 (UNetModel.__init__) and
code/nn.py:139-184 / 241-254 (ResBlock / AttentionBlock parameters) so that
`state_dict_spec()` yields exactly the reference's `state_dict()` keys and shapes, in order.
The HIP library builds its own execution plan from the same hyper-parameters
(csrc/unet_plan.hip); tests check both agree.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class UNetConfig:
    """Hyper-parameters hard-coded in create_model_and_diffusion (code/train_inpainting.py:208-224)."""
    image_size: int = 256
    in_channels: int = 9
    model_channels: int = 128
    out_channels: int = 6
    num_res_blocks: int = 1
    attention_resolutions: tuple = (16,)
    channel_mult: tuple = (1, 1, 2, 2, 4, 4)
    num_head_channels: int = 64
    use_scale_shift_norm: bool = True
    resblock_updown: bool = True

    def as_dict(self):
        return asdict(self)


FULL = UNetConfig()
REDUCED = UNetConfig(image_size=64, model_channels=64)


def _res_params(p, cin, cout, emb):
    out = [
        (p + "in_layers.0.weight", (cin,)), (p + "in_layers.0.bias", (cin,)),
        (p + "in_layers.2.weight", (cout, cin, 3, 3)), (p + "in_layers.2.bias", (cout,)),
        (p + "emb_layers.1.weight", (2 * cout, emb)), (p + "emb_layers.1.bias", (2 * cout,)),
        (p + "out_layers.0.weight", (cout,)), (p + "out_layers.0.bias", (cout,)),
        (p + "out_layers.3.weight", (cout, cout, 3, 3)), (p + "out_layers.3.bias", (cout,)),
    ]
    if cin != cout:
        out += [(p + "skip_connection.weight", (cout, cin, 1, 1)), (p + "skip_connection.bias", (cout,))]
    return out


def _attn_params(p, c):
    return [
        (p + "norm.weight", (c,)), (p + "norm.bias", (c,)),
        (p + "qkv.weight", (3 * c, c, 1)), (p + "qkv.bias", (3 * c,)),
        (p + "proj_out.weight", (c, c, 1)), (p + "proj_out.bias", (c,)),
    ]


def layer_plan(cfg: UNetConfig = FULL):
    """Ordered blocks: list of (section, block_index, [layers]); layer = dict(kind, prefix, cin, cout, res).

    `res` is the spatial size at the layer's input. kinds: conv_in, res, res_down, res_up, attn, out.
    """
    mc = cfg.model_channels
    emb = 4 * mc
    res = cfg.image_size
    ch = int(cfg.channel_mult[0] * mc)
    blocks = [("input", 0, [dict(kind="conv_in", prefix="input_blocks.0.0.", cin=cfg.in_channels, cout=ch, res=res)])]
    chans = [ch]
    ds = 1
    nlev = len(cfg.channel_mult)
    for level, mult in enumerate(cfg.channel_mult):
        for _ in range(cfg.num_res_blocks):
            i = len(blocks)
            out = int(mult * mc)
            layers = [dict(kind="res", prefix=f"input_blocks.{i}.0.", cin=ch, cout=out, res=res)]
            ch = out
            if ds in cfg.attention_resolutions:
                layers.append(dict(kind="attn", prefix=f"input_blocks.{i}.1.", cin=ch, cout=ch, res=res))
            blocks.append(("input", i, layers))
            chans.append(ch)
        if level != nlev - 1:
            i = len(blocks)
            blocks.append(("input", i, [dict(kind="res_down", prefix=f"input_blocks.{i}.0.", cin=ch, cout=ch, res=res)]))
            chans.append(ch)
            ds *= 2
            res //= 2
    blocks.append(("middle", 0, [
        dict(kind="res", prefix="middle_block.0.", cin=ch, cout=ch, res=res),
        dict(kind="attn", prefix="middle_block.1.", cin=ch, cout=ch, res=res),
        dict(kind="res", prefix="middle_block.2.", cin=ch, cout=ch, res=res),
    ]))
    j = 0
    for level, mult in list(enumerate(cfg.channel_mult))[::-1]:
        for i in range(cfg.num_res_blocks + 1):
            ich = chans.pop()
            out = int(mc * mult)
            layers = [dict(kind="res", prefix=f"output_blocks.{j}.0.", cin=ch + ich, cout=out, res=res, skip_ch=ich)]
            ch = out
            if ds in cfg.attention_resolutions:
                layers.append(dict(kind="attn", prefix=f"output_blocks.{j}.1.", cin=ch, cout=ch, res=res))
            if level and i == cfg.num_res_blocks:
                layers.append(dict(kind="res_up", prefix=f"output_blocks.{j}.{len(layers)}.", cin=ch, cout=ch, res=res))
                ds //= 2
                res *= 2
            blocks.append(("output", j, layers))
            j += 1
    blocks.append(("out", 0, [dict(kind="out", prefix="out.", cin=ch, cout=cfg.out_channels, res=res)]))
    return blocks


def state_dict_spec(cfg: UNetConfig = FULL, prefix: str = "base_model."):
    """(key, shape) for every parameter of DiffusionInpaintingModel, in state_dict order."""
    mc = cfg.model_channels
    emb = 4 * mc
    spec = [("time_embed.0.weight", (emb, mc)), ("time_embed.0.bias", (emb,)),
            ("time_embed.2.weight", (emb, emb)), ("time_embed.2.bias", (emb,))]
    for section, _, layers in layer_plan(cfg):
        for L in layers:
            p, k = L["prefix"], L["kind"]
            if k == "conv_in":
                spec += [(p + "weight", (L["cout"], L["cin"], 3, 3)), (p + "bias", (L["cout"],))]
            elif k in ("res", "res_down", "res_up"):
                spec += _res_params(p, L["cin"], L["cout"], emb)
            elif k == "attn":
                spec += _attn_params(p, L["cin"])
            elif k == "out":
                spec += [("out.0.weight", (L["cin"],)), ("out.0.bias", (L["cin"],)),
                         ("out.2.weight", (L["cout"], L["cin"], 3, 3)), ("out.2.bias", (L["cout"],))]
    return [(prefix + k, s) for k, s in spec]


def gflop_per_image(cfg: UNetConfig = FULL):
    """Algorithmic 2*MAC FLOPs of one UNet eval for one image (388.84 at FULL)."""
    f = 0.0
    for _, _, layers in layer_plan(cfg):
        for L in layers:
            r, cin, cout = L["res"], L["cin"], L["cout"]
            if L["kind"] == "conv_in" or L["kind"] == "out":
                f += 2 * r * r * 9 * cin * cout
            elif L["kind"] in ("res", "res_down", "res_up"):
                ro = r // 2 if L["kind"] == "res_down" else (r * 2 if L["kind"] == "res_up" else r)
                f += 2 * ro * ro * 9 * cin * cout + 2 * ro * ro * 9 * cout * cout
                if cin != cout:
                    f += 2 * ro * ro * cin * cout
            elif L["kind"] == "attn":
                T = r * r
                c = cin
                f += 2 * T * c * 3 * c + 2 * T * c * c + 2 * 2 * T * T * c
    mc = cfg.model_channels
    f += 2 * (mc * 4 * mc + 16 * mc * mc)
    return f / 1e9
