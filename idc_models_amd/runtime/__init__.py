"""MI355X execution runtime: model lowering -> static plan -> HIP-graph replay."""
from .program import FusedProgram, FusedStep, fused_supported

__all__ = ["FusedProgram", "FusedStep", "fused_supported"]
