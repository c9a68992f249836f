"""MI355X GPU attribution: amd-smi telemetry, HBM-vs-host OOM scoring, RCCL/xGMI rank topology."""
