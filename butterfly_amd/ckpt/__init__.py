"""Checkpoints: sharded safetensors + manifest (butterfly-ckpt v1), resharding, HF import."""
from .format import load_into, model_config, read_manifest, reshard, save  # noqa: F401
