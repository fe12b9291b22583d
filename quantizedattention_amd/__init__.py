"""quantizedattention_amd — MI355X (gfx950) quantized fused attention.

Drop-in modules mirroring selau642/QuantizedAttention:
  quantizedattention_amd.attention_bf16, .attention_int8, .attention_jvp
Head-sharded multi-GPU wrapper: quantizedattention_amd.sharded
"""
__version__ = "0.1.0"
