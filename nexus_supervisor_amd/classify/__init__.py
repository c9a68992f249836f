"""Failure classification (reference event table + pod/job status + GPU rules)."""
from . import reference_rules
from .classifier import (
    DECIDED,
    EVIDENCE,
    IGNORED,
    NOOP,
    STALE,
    Classifier,
    EvidenceBook,
    ObjectLookup,
    render_trace,
)

__all__ = ["reference_rules", "DECIDED", "EVIDENCE", "IGNORED", "NOOP", "STALE", "Classifier",
           "EvidenceBook", "ObjectLookup", "render_trace"]
