"""sparkglm_amd -- MI355X-native fitting engine for sparkGLM's lm()/glm() hot path."""
from ._lib import IllegalArgumentException, MatrixSingularException, SGLMError  # noqa: F401
from .engine import Engine, FitGLM, FitLM, device_count  # noqa: F401

__version__ = "0.1.0"
