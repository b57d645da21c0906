"""Serving: KV-cache generation for the Llama decoder (beyond the training-only reference)."""
from .generator import ContinuousBatcher, Generator, Request

__all__ = ["ContinuousBatcher", "Generator", "Request"]
