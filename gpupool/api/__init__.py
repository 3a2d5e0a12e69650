"""API surface of the gpupool operator: schema source, OpenAPI checks and condition helpers."""
from . import schema  # noqa: F401
