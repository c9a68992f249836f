"""The per-request lifecycle row ``nexus.checkpoints`` and lifecycle stages.

Schema is byte-compatible with ``/root/reference/test-resources/checkpoints.cql:1-29``
(19 columns, composite partition key ``((algorithm, id))``, three secondary
indexes).  The Python model mirrors nexus-core ``models.CheckpointedRequest``
(used at ``/root/reference/services/supervisor.go:264-370``).

Stage strings other than BUFFERED / RUNNING / CANCELLED (seen in the seed data,
``checkpoints.cql:35,44,98``) cannot be verified offline, so they and
the finished set are configuration (``stages:`` section, :class:`..config.schema.StagesConfig`)
applied process-wide by :func:`configure_lifecycle_stages` — every supervisor and
shard-worker process applies its config's section at construction.  Readers go
through the class attributes / :func:`finished_stages` at call time, never through a
copy taken at import.
"""
from __future__ import annotations

import copy
import datetime as _dt
from dataclasses import dataclass, fields
from typing import Dict, Iterable, Optional, Tuple


class LifecycleStage:
    NEW = "NEW"
    BUFFERED = "BUFFERED"
    RUNNING = "RUNNING"
    COMPLETED = "COMPLETED"
    FAILED = "FAILED"
    SCHEDULING_FAILED = "SCHEDULING_FAILED"
    DEADLINE_EXCEEDED = "DEADLINE_EXCEEDED"
    CANCELLED = "CANCELLED"


DEFAULT_STAGES: Dict[str, str] = {a: getattr(LifecycleStage, a) for a in vars(LifecycleStage) if a.isupper()}
# nexus-core ``CheckpointedRequest.IsFinished()``: proven for CANCELLED
# (/root/reference/services/supervisor_test.go:473-540), presumed for terminal stages.
TERMINAL_ATTRS = ("COMPLETED", "FAILED", "SCHEDULING_FAILED", "DEADLINE_EXCEEDED", "CANCELLED")
UNFINISHED_ATTRS = ("NEW", "BUFFERED", "RUNNING")


def _terminal_set() -> frozenset:
    return frozenset(getattr(LifecycleStage, a) for a in TERMINAL_ATTRS)


FINISHED_STAGES = _terminal_set()


def finished_stages() -> frozenset:
    """The current finished set (reads the module state at call time)."""
    return FINISHED_STAGES


def unfinished_stages() -> Tuple[str, ...]:
    """Stages a run can still leave: the conditional-write guard (``IF lifecycle_stage IN``)."""
    return tuple(s for s in (getattr(LifecycleStage, a) for a in UNFINISHED_ATTRS) if s not in FINISHED_STAGES)


def configure_lifecycle_stages(mapping: Optional[Dict[str, str]] = None, finished: Optional[Iterable[str]] = None) -> None:
    """Set the stage strings (``{"FAILED": "FAILED_V2", ...}``, attributes not named keep
    their defaults) and the finished set.  ``finished`` None rebuilds the set from the
    terminal attributes, so remapping only ``FAILED`` moves it in the set too."""
    global FINISHED_STAGES
    mapping = dict(mapping or {})
    for attr in mapping:
        if attr not in DEFAULT_STAGES:
            raise KeyError(attr)
    for attr, default in DEFAULT_STAGES.items():
        setattr(LifecycleStage, attr, mapping.get(attr) or default)
    FINISHED_STAGES = frozenset(finished) if finished else _terminal_set()


KEYSPACE = "nexus"
TABLE = "checkpoints"

# (column, cql type) in table order — checkpoints.cql:3-21
COLUMNS: Tuple[Tuple[str, str], ...] = (
    ("algorithm", "text"),
    ("id", "text"),
    ("lifecycle_stage", "text"),
    ("payload_uri", "text"),
    ("result_uri", "text"),
    ("algorithm_failure_cause", "text"),
    ("algorithm_failure_details", "text"),
    ("received_by_host", "text"),
    ("received_at", "timestamp"),
    ("sent_at", "timestamp"),
    ("applied_configuration", "text"),
    ("configuration_overrides", "text"),
    ("content_hash", "text"),
    ("last_modified", "timestamp"),
    ("tag", "text"),
    ("api_version", "text"),
    ("job_uid", "text"),
    ("parent", "text"),
    ("payload_valid_for", "text"),
)
COLUMN_NAMES = tuple(c for c, _ in COLUMNS)
PARTITION_KEY = ("algorithm", "id")
SECONDARY_INDEXES = (("submission_tag", "tag"), ("host", "received_by_host"), ("lifecycle_stage", "lifecycle_stage"))
# Columns this supervisor owns: the owned-columns UPDATE writes only these.
OWNED_COLUMNS = ("lifecycle_stage", "algorithm_failure_cause", "algorithm_failure_details", "last_modified")


def create_table_cql(keyspace: str = KEYSPACE, table: str = TABLE) -> str:
    cols = ",\n".join(f"    {n:<25} {t}" for n, t in COLUMNS)
    return f"create table {keyspace}.{table}\n(\n{cols},\n    PRIMARY KEY ((algorithm, id))\n);"


def create_index_cql(keyspace: str = KEYSPACE, table: str = TABLE) -> Tuple[str, ...]:
    return tuple(f"create index {name} ON {keyspace}.{table} ({col});" for name, col in SECONDARY_INDEXES)


def utcnow() -> _dt.datetime:
    return _dt.datetime.now(_dt.timezone.utc)


@dataclass
class CheckpointedRequest:
    """One row of ``nexus.checkpoints``. ``timestamp`` columns are aware UTC datetimes."""

    algorithm: str = ""
    id: str = ""
    lifecycle_stage: Optional[str] = None
    payload_uri: Optional[str] = None
    result_uri: Optional[str] = None
    algorithm_failure_cause: Optional[str] = None
    algorithm_failure_details: Optional[str] = None
    received_by_host: Optional[str] = None
    received_at: Optional[_dt.datetime] = None
    sent_at: Optional[_dt.datetime] = None
    applied_configuration: Optional[str] = None
    configuration_overrides: Optional[str] = None
    content_hash: Optional[str] = None
    last_modified: Optional[_dt.datetime] = None
    tag: Optional[str] = None
    api_version: Optional[str] = None
    job_uid: Optional[str] = None
    parent: Optional[str] = None
    payload_valid_for: Optional[str] = None

    def is_finished(self) -> bool:
        return self.lifecycle_stage in FINISHED_STAGES

    def deep_copy(self) -> "CheckpointedRequest":
        return copy.copy(self)  # all fields are immutable scalars

    @property
    def key(self) -> Tuple[str, str]:
        return (self.algorithm, self.id)

    def as_row(self) -> Tuple:
        return tuple(getattr(self, n) for n in COLUMN_NAMES)

    @classmethod
    def from_row(cls, row) -> "CheckpointedRequest":
        if isinstance(row, dict):
            return cls(**{n: row.get(n) for n in COLUMN_NAMES})
        return cls(*row)

    def to_dict(self) -> Dict[str, object]:
        return {f.name: getattr(self, f.name) for f in fields(self)}


class StageRow:
    """The projected stage read (``SELECT lifecycle_stage``) of the owned-columns path: the
    key and the stage, every other column None.  One per decision, so it is a three-slot
    object instead of the 19-field dataclass (whose generated ``__init__`` was ~1 % of a
    shard worker's CPU)."""

    __slots__ = ("algorithm", "id", "lifecycle_stage")

    def __init__(self, algorithm: str, id: str, lifecycle_stage: Optional[str]):  # noqa: A002 - the column name
        self.algorithm = algorithm
        self.id = id
        self.lifecycle_stage = lifecycle_stage

    def __getattr__(self, name: str):
        if name in _OTHER_COLUMNS:
            return None
        raise AttributeError(name)

    def is_finished(self) -> bool:
        return self.lifecycle_stage in FINISHED_STAGES

    @property
    def key(self) -> Tuple[str, str]:
        return (self.algorithm, self.id)

    def deep_copy(self) -> CheckpointedRequest:
        return CheckpointedRequest(self.algorithm, self.id, self.lifecycle_stage)


_OTHER_COLUMNS = frozenset(n for n in COLUMN_NAMES if n not in ("algorithm", "id", "lifecycle_stage"))
