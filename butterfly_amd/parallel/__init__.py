"""Parallelism: device mesh, communicator (RCCL / gloo), pipeline and expert parallel helpers."""
from .comm import Communicator, init_distributed  # noqa: F401
from .mesh import Mesh  # noqa: F401
