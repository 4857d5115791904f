"""Model zoo: Llama / Qwen3 / Qwen3-MoE / Mixtral transformers, GPT-MoE, attention variants, LeNet."""
from .config import ModelConfig, get_model_config, registered_models
from .transformer import (MLP, Attention, DecoderLayer, TransformerLM, build_model, stage_layer_range)

__all__ = ["ModelConfig", "get_model_config", "registered_models", "MLP", "Attention", "DecoderLayer",
           "TransformerLM", "build_model", "stage_layer_range"]
