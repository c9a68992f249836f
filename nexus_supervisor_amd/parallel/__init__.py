"""Concurrency: keyed rate-limited work pipeline, token bucket, backoff."""
