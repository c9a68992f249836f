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


class NotFound(ApiError):
    pass


class Conflict(ApiError):
    pass


class Gone(ApiError):
    pass


def from_status(status: int, body: Optional[Dict[str, Any]] = None) -> ApiError:
    body = body or {}
    reason = body.get("reason", "") if isinstance(body, dict) else ""
    message = body.get("message", "") if isinstance(body, dict) else str(body)
    cls = {404: NotFound, 409: Conflict, 410: Gone}.get(status, ApiError)
    return cls(status, reason, message, body if isinstance(body, dict) else None)
