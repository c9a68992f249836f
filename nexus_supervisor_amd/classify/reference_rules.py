"""R-EVT: the reference decision table, byte-exact.

Source: ``/root/reference/services/supervisor.go:159-258`` (table in SURVEY
§2.9.1).  The RunStatusMessage strings below are the exact literals of
``supervisor.go:176,187,198``; pod-side messages are the event reason itself
(``:227,237,247``).
"""
from __future__ import annotations

from ..models.decisions import DecisionAction as A
from ..models.decisions import FailureClass as F

MSG_FAILED_CREATE = "Unable to launch a container for the algorithm - please review configuration and try again."
MSG_DEADLINE = "Algorithm exceeded its max allowed run time limit or retry attempt count."
MSG_FATAL = "Algorithm encountered a fatal error during execution."

# Job-kind event reason -> (action, message, failure class)
JOB_EVENT_RULES = {
    "FailedCreate": (A.TO_FAIL_STUCK_IN_PENDING, MSG_FAILED_CREATE, F.SCHEDULING),
    "DeadlineExceeded": (A.TO_FAIL_DEADLINE_EXCEEDED, MSG_DEADLINE, F.DEADLINE),
    "BackoffLimitExceeded": (A.TO_FAIL_DEADLINE_EXCEEDED, MSG_DEADLINE, F.BACKOFF_LIMIT),
    "PodFailurePolicy": (A.TO_FAIL_FATAL_ERROR, MSG_FATAL, F.FATAL),
}

# Pod-kind event reason -> (action, failure class); message = reason (supervisor.go:227,237,247)
POD_EVENT_RULES = {
    "Started": (A.TO_RUNNING, F.NONE),
    "Failed": (A.TO_FAIL_STUCK_IN_PENDING, F.SCHEDULING),
    "BackOff": (A.TO_FAIL_FATAL_ERROR, F.FATAL),
}

# Actuation prefixes (supervisor.go:298,325); DEADLINE has no prefix (:350).
CAUSE_PREFIX = {
    A.TO_FAIL_STUCK_IN_PENDING: "Algorithm submission was buffered, but failed to launch on the target cluster: ",
    A.TO_FAIL_FATAL_ERROR: "Algorithm encountered a fatal error during execution: ",
    A.TO_FAIL_DEADLINE_EXCEEDED: "",
}


def failure_cause(action: str, run_status_message: str, doubled_fatal_cause: bool = True) -> str:
    """``algorithm_failure_cause`` for a failing action.

    With ``doubled_fatal_cause`` (reference behaviour) a Job ``PodFailurePolicy``
    yields "Algorithm encountered a fatal error during execution: Algorithm
    encountered a fatal error during execution." (SURVEY §2.9.2); otherwise the
    duplicated sentence is collapsed.
    """
    prefix = CAUSE_PREFIX[action]
    if not doubled_fatal_cause and action == A.TO_FAIL_FATAL_ERROR and run_status_message == MSG_FATAL:
        return MSG_FATAL
    return prefix + run_status_message
