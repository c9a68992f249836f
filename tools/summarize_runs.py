"""Median and range of bench lines (the numbers README / BASELINE quote).

    python tools/summarize_runs.py profiles/r4_final/bench_*.json [...]

Each file holds bench.py's output; its last line is the JSON result.  Prints, per metric,
``median [min – max] (n)``: failures/s, replica CPU per failure, saturated p50 / p99, the
open-loop probe's p50 / p99, and whether any run was harness-bound or wrong."""
import glob
import json
import statistics
import sys


def _last_json(path):
    with open(path) as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip().startswith("{")]
    return json.loads(lines[-1]) if lines else None


def rows(paths):
    out = []
    for p in paths:
        d = _last_json(p)
        if not d:
            continue
        la = d.get("latency_at_rate") or {}
        out.append({"file": p, "value": d["value"], "cpu_us": d.get("supervisor_cpu_us_per_event_rank0"),
                    "sat_p50": d.get("p50_ms"), "sat_p99": d.get("p99_ms"), "probe_p50": la.get("p50_ms"),
                    "probe_p99": la.get("p99_ms"), "bound": (d.get("harness_bound") or {}).get("bound"),
                    "wrong": d.get("wrong_stage", 0) + ((d.get("readback") or {}).get("wrong") or 0),
                    "shape": (d.get("config") or {}).get("hbm_oom_shape")})
    return out


def summary(rs):
    def band(key):
        vals = [r[key] for r in rs if r.get(key) is not None]
        if not vals:
            return None
        return {"median": round(statistics.median(vals), 3), "min": min(vals), "max": max(vals), "n": len(vals)}

    return {k: band(k) for k in ("value", "cpu_us", "sat_p50", "sat_p99", "probe_p50", "probe_p99")} | {
        "harness_bound_runs": sum(1 for r in rs if r["bound"]), "wrong": sum(r["wrong"] for r in rs),
        "shapes": sorted({r["shape"] for r in rs if r["shape"]})}


def main(argv=None) -> int:
    paths = []
    for a in (argv if argv is not None else sys.argv[1:]):
        paths += sorted(glob.glob(a))
    rs = rows(paths)
    for r in rs:
        print(f"{r['file']}: {r['value']:.0f}/s {r['cpu_us']} µs  sat {r['sat_p50']}/{r['sat_p99']} ms  "
              f"probe {r['probe_p50']}/{r['probe_p99']} ms")
    s = summary(rs)
    for k in ("value", "cpu_us", "sat_p50", "sat_p99", "probe_p50", "probe_p99"):
        b = s[k]
        if b:
            print(f"{k:10s} median {b['median']}  [{b['min']} – {b['max']}]  (n={b['n']})")
    print(f"harness-bound runs {s['harness_bound_runs']}, wrong stages/rows {s['wrong']}, shapes {s['shapes']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
