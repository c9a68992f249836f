"""Config 3a: GPU attribution through the deployed path — the node agent as its own process
(``python -m nexus_supervisor_amd agent``) annotating failed pods, the supervisor without
local telemetry holding their decisions up to ``gpu.evidence-wait`` for the annotation.

The Job of a failed default pod reports ``BackoffLimitExceeded`` on its own watch stream
while the pod's decision is held for the agent: the Job decision must wait for the same
evidence, or it writes DEADLINE_EXCEEDED with no GPU ahead of the annotation (the HBM-OOM
rewrite of ``rules.oom-fails-backoff-job`` never sees the OOM).  The GPU run of this
scenario is ``tests/test_gpu_box.py::test_cfg3a_agent_path_real_hbm_oom``.
"""
from nexus_supervisor_amd.bench.scenarios import cfg3_agent


def test_agent_process_attributes_default_pods_within_the_wait(arun):
    r = arun(cfg3_agent("uncapped", runs=4, gpu=False), timeout=240)
    assert r["acked"] == 4 and r["wrong"] == 0, r
    # every pod was held for the annotation and every one landed before the wait ran out
    assert r["deferred_for_gpu_evidence"] == 4 and r["evidence_wait_expired"] == 0, r
    # the Job's BackoffLimitExceeded waited for the pod's evidence instead of writing first
    assert r["job_decisions_awaited_evidence"] >= 1, r
    # the agent read the container log from the node: no pods/log read by the supervisor
    assert r["supervisor_pod_log_reads"] == 0, r
    assert r["p99_ms"] < 2000, r  # well inside the 2 s evidence wait
    assert r["agent_annotations"] == 4, r  # one annotation PATCH per failed pod
    # every row carries the agent's GPU record, whichever decision (pod's or Job's) wrote it
    assert r["rows_with_gpu_record"] == 4, r
