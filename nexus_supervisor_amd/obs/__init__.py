"""Observability: klog-style JSON logs, metrics (Prometheus + DogStatsD), latency histograms, profiling, HTTP endpoints."""
