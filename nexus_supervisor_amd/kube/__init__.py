"""Kubernetes API access: REST/watch client and API errors."""
