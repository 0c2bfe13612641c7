"""Encoder registry (reference src/model/encoder/__init__.py:7-18)."""
from .encoder import Encoder
from .encoder_trans import EncoderTrans, EncoderTransCfg

ENCODERS = {"trans": (EncoderTrans, None)}

EncoderCfg = EncoderTransCfg


def get_encoder(cfg: EncoderCfg):
    encoder, visualizer = ENCODERS[cfg.name]
    encoder = encoder(cfg)
    return encoder, visualizer


__all__ = ["ENCODERS", "Encoder", "EncoderCfg", "EncoderTrans", "EncoderTransCfg", "get_encoder"]
