"""Kubernetes API errors (``metav1.Status`` failures)."""
from __future__ import annotations

from typing import Any, Dict, Optional


class ApiError(Exception):
    def __init__(self, status: int, reason: str = "", message: str = "", body: Optional[Dict[str, Any]] = None):
        super().__init__(f"{status} {reason}: {message}".strip())
        self.status = status
        self.reason = reason
        self.message = message
        self.body = body or {}
        self.retry_after: Optional[float] = None  # the server's Retry-After hint, seconds


class NotFound(ApiError):
    pass


class Conflict(ApiError):
    pass


class Gone(ApiError):
    pass


class TooManyRequests(ApiError):
    """429 (API Priority and Fairness rejected the request, or a max-in-flight limit)."""


def from_status(status: int, body: Optional[Dict[str, Any]] = None, retry_after: Optional[float] = None) -> ApiError:
    """The typed error of a failed answer; ``retry_after`` = the server's ``Retry-After``
    hint in seconds (kept on every error: a 503 may carry one too)."""
    body = body or {}
    reason = body.get("reason", "") if isinstance(body, dict) else ""
    message = body.get("message", "") if isinstance(body, dict) else str(body)
    cls = {404: NotFound, 409: Conflict, 410: Gone, 429: TooManyRequests}.get(status, ApiError)
    err = cls(status, reason, message, body if isinstance(body, dict) else None)
    err.retry_after = retry_after
    return err
