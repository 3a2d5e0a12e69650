"""In-repo kube-apiserver simulator (the envtest/kind stand-in)."""
from .store import ApiError, ResourceType, Store  # noqa: F401
