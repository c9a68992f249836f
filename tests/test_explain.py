"""``python -m nexus_supervisor_amd explain``: offline decisions for kubectl JSON — the
reference scenarios' stages and byte-exact causes, and an HBM-OOM attributed to its
physical GPU from the node agent's annotation."""
import json
import os
import subprocess
import sys

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.explain import explain, parse_objects
from nexus_supervisor_amd.testing.seed import make_pod, reference_scenarios

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg():
    return load_config(path=None, env={}, overrides={})


def test_parse_objects_lists_and_streams():
    pod = make_pod("a", _cfg().labels)
    pod.pop("kind")
    text = json.dumps({"kind": "PodList", "items": [pod]}) + "\n" + json.dumps(
        {"kind": "List", "items": [{"kind": "Job", "metadata": {"name": "j"}}, {"kind": "Secret"}]})
    got = parse_objects(text)
    assert [o["kind"] for o in got] == ["Pod", "Job"] and got[0]["metadata"]["name"] == "a-acdey"


def test_reference_scenarios_explained():
    """Each reference scenario's objects (supervisor_test.go:46-540) → the stage the
    reference test expects, with its byte-exact cause; the CANCELLED run's Started event
    is a RUNNING decision (explain does not read the store: the supervisor skips it as
    finished)."""
    for s in reference_scenarios():
        out = explain(s.objects, _cfg())
        decided = {d["request_id"]: d for rec in out for d in rec.get("decisions", ())}
        for rid, stage in s.expected.items():
            if stage == "CANCELLED":
                assert decided[rid]["lifecycle_stage"] == "RUNNING"
                continue
            assert decided[rid]["lifecycle_stage"] == stage, (s.name, decided)
            if stage != "RUNNING":
                assert decided[rid]["delete_job"] and decided[rid]["algorithm_failure_cause"]
    pfp = next(s for s in reference_scenarios() if s.name == "pod-failure-policy-oom")
    d = [d for rec in explain(pfp.objects, _cfg()) for d in rec.get("decisions", ())][0]
    assert d["algorithm_failure_cause"] == ("Algorithm encountered a fatal error during execution: "
                                            "Algorithm encountered a fatal error during execution.")


def test_hbm_oom_pod_explained_with_gpu_and_signals(tmp_path):
    msg = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 8.00 GiB. GPU 3 has a total capacity of "
           "287.98 GiB of which 2.10 GiB is free.")
    ev = {"source": "agent", "gpus": [
        {"index": 7, "vram_total_mb": 294896, "vram_peak_mb": 292000, "proc_peak_vram_bytes": 280 << 30,
         "procs": [{"pid": 4242, "rank": 3, "local_rank": 3}]}]}
    pod = make_pod("oom-run", _cfg().labels, gpus=4, rv="2", env={"HIP_VISIBLE_DEVICES": "4,5,6,7", "LOCAL_RANK": "3"},
                   status={"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                       "terminated": {"reason": "Error", "exitCode": 1, "message": msg}}}]},
                   annotations={"nexus.amd.com/gpu-evidence": json.dumps(ev)})
    f = tmp_path / "pod.json"
    f.write_text(json.dumps({"kind": "List", "items": [pod]}))
    p = subprocess.run([sys.executable, "-m", "nexus_supervisor_amd", "explain", str(f)], cwd=str(tmp_path),
                       capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=ROOT, NEXUS__CQL_STORE_TYPE="memory"))
    assert p.returncode == 0, p.stderr
    out = json.loads(p.stdout)
    d = out[0]["decisions"][0]
    assert out[0]["status"] == "decided" and d["lifecycle_stage"] == "FAILED" and d["failure_class"] == "hbm-oom"
    assert d["oom"]["gpu_index"] == 7 and d["oom"]["gpu_logical_index"] == 3
    assert any("HIP OOM signature" in s for s in d["oom"]["signals"])
    assert json.loads(d["algorithm_failure_details"])["class"] == "hbm-oom"
