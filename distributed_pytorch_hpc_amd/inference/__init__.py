"""Serving: KV-cache generation for the Llama decoder (beyond the training-only reference)."""
from .generator import Generator

__all__ = ["Generator"]
