"""The per-request lifecycle row ``nexus.checkpoints`` and lifecycle stages.

Schema is byte-compatible with ``/root/reference/test-resources/checkpoints.cql:1-29``
(19 columns, composite partition key ``((algorithm, id))``, three secondary
indexes).  The Python model mirrors nexus-core ``models.CheckpointedRequest``
(used at ``/root/reference/services/supervisor.go:264-370``).

Stage strings other than BUFFERED / RUNNING / CANCELLED (seen in the seed data,
``checkpoints.cql:35,44,98``) cannot be verified offline; they are
plain module constants so a deployment can pin them via
:func:`configure_lifecycle_stages`.
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


# nexus-core ``CheckpointedRequest.IsFinished()``: proven for CANCELLED
# (/root/reference/services/supervisor_test.go:473-540), presumed for terminal stages.
FINISHED_STAGES = frozenset(
    {
        LifecycleStage.COMPLETED,
        LifecycleStage.FAILED,
        LifecycleStage.SCHEDULING_FAILED,
        LifecycleStage.DEADLINE_EXCEEDED,
        LifecycleStage.CANCELLED,
    }
)


def configure_lifecycle_stages(mapping: Dict[str, str], finished: Optional[Iterable[str]] = None) -> None:
    """Override stage strings (``{"FAILED": "FAILED_V2", ...}``) and the finished set."""
    global FINISHED_STAGES
    for attr, value in mapping.items():
        if not hasattr(LifecycleStage, attr):
            raise KeyError(attr)
        setattr(LifecycleStage, attr, value)
    if finished is not None:
        FINISHED_STAGES = frozenset(finished)


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
