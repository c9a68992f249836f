"""Domain models: checkpoint row + lifecycle stages, decisions, slim K8s object views."""
from .checkpoint import (
    COLUMN_NAMES,
    COLUMNS,
    OWNED_COLUMNS,
    CheckpointedRequest,
    LifecycleStage,
    configure_lifecycle_stages,
    create_index_cql,
    finished_stages,
    unfinished_stages,
    create_table_cql,
    utcnow,
)
from .decisions import Decision, DecisionAction, FailureClass, RunStatusAnalysisResult

__all__ = [
    "COLUMN_NAMES", "COLUMNS", "OWNED_COLUMNS", "CheckpointedRequest", "LifecycleStage",
    "configure_lifecycle_stages", "create_index_cql", "create_table_cql", "finished_stages", "unfinished_stages", "utcnow",
    "Decision", "DecisionAction", "FailureClass", "RunStatusAnalysisResult",
]
