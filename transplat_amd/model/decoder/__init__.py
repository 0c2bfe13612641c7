"""Decoder registry (reference src/model/decoder/__init__.py:5-13).

`splatting_hip` is the gfx950 rasterizer; the reference name `splatting_cuda` maps to the same
class so an unchanged reference config selects it.
"""
from .decoder import DatasetCfgLite, Decoder, DecoderOutput
from .decoder_splatting_hip import DecoderSplattingHIP, DecoderSplattingHIPCfg

DECODERS = {
    "splatting_hip": DecoderSplattingHIP,
    "splatting_cuda": DecoderSplattingHIP,
}

DecoderCfg = DecoderSplattingHIPCfg


def get_decoder(decoder_cfg: DecoderCfg, dataset_cfg) -> Decoder:
    return DECODERS[decoder_cfg.name](decoder_cfg, dataset_cfg)


__all__ = ["DECODERS", "DatasetCfgLite", "Decoder", "DecoderOutput", "DecoderSplattingHIP",
           "DecoderSplattingHIPCfg", "get_decoder"]
