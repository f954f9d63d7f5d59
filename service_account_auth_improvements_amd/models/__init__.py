"""Model families of the worker runtime."""
from .llama import Llama, LlamaConfig  # noqa: F401
