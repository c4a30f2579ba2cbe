"""mep_amd -- MI355X-native (gfx950) drop-in for the tri-modal residual-attention training path
of youngzhou97qz/Multimodal-emotion-processing.

Public surface (mirrors the reference scripts):
  mep_amd.cmu_mosei   Concat_Trans, Multi_ATTN, Attention_Block, Unify_Dimension,
                      multi_circle_loss, train, valid, run, get_parameter_number
  mep_amd.ren_mme     Base_model (+ Ren-MME variants of the same classes), multi_loss, train, valid
  mep_amd.optim       FusedAdamW / FusedAdam (clip + update over the flat parameter buffer)
  mep_amd.engine      TrainEngine (graph-captured fused step, RCCL data parallel)
Kernels: libmep_hip.so (csrc/, C ABI in include/mep.h).  No CPU fallback.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
__version__ = '0.1.0'


def library_path():
    return os.path.join(PKG_DIR, 'libmep_hip.so')
