from .mesh import Mesh, init_mesh, shutdown
from .schedule import Schedule, build_schedule, KINDS
from .pipeline import PipelineEngine, StepResult, split_sizes

__all__ = ["Mesh", "init_mesh", "shutdown", "Schedule", "build_schedule", "KINDS", "PipelineEngine",
           "StepResult", "split_sizes"]
