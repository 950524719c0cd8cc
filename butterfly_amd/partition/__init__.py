"""Model partitioning: cost model, (dp, tp, pp, ep) + cut-point search, PartitionPlan format."""
from .costmodel import CostModel  # noqa: F401
from .hw import MI355X, Hardware  # noqa: F401
from .plan import PartitionPlan, ShardSpec  # noqa: F401
from .search import evaluate, factorizations, partition  # noqa: F401
