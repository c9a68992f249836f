"""Typed configuration schema.

Reference keys are kept byte-identical (``/root/reference/app/app_config.go:8-25``;
``/root/reference/appconfig.local.yaml:1-19``).  Defaults equal the Helm chart
defaults (``/root/reference/.helm/values.yaml:119-165``) instead of Go's zero
values, so an empty ``workers: ""`` no longer silently means zero workers
(SURVEY §5.6).  Everything under a key the reference does not have is an
extension of this build and documented in ``docs/CONFIG.md``.

Each dataclass field carries ``metadata={"key": "<kebab-key>"}``; durations are
float seconds tagged ``"kind": "duration"``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List


def _k(key: str, kind: str | None = None, **extra):
    md = {"key": key}
    if kind:
        md["kind"] = kind
    md.update(extra)
    return md


CQL_STORE_ASTRA = "astra"
CQL_STORE_SCYLLA = "scylla"
CQL_STORE_MEMORY = "memory"  # extension: in-process store for tests / dry runs
CQL_STORE_TYPES = (CQL_STORE_ASTRA, CQL_STORE_SCYLLA, CQL_STORE_MEMORY)


@dataclass
class AstraBundleConfig:
    """``request.AstraBundleConfig`` (``/root/reference/appconfig.local.yaml:1-4``)."""

    # Astra secure-connect zip, base64
    secure_connection_bundle_base64: str = field(default="", metadata=_k("secure-connection-bundle-base64", secret=True))
    gateway_user: str = field(default="", metadata=_k("gateway-user"))  # Astra token client id
    gateway_password: str = field(default="", metadata=_k("gateway-password", secret=True))  # Astra token secret
    # extensions
    keyspace: str = field(default="nexus", metadata=_k("keyspace"))  # keyspace of the checkpoints table
    table: str = field(default="checkpoints", metadata=_k("table"))  # checkpoints table (nexus-core schema)
    # consistency of reads and writes; conditional writes use the matching SERIAL level
    consistency: str = field(default="LOCAL_QUORUM", metadata=_k("consistency"))
    request_timeout: float = field(default=5.0, metadata=_k("request-timeout", "duration"))  # per CQL request


@dataclass
class ScyllaCqlStoreConfig:
    """``request.ScyllaCqlStoreConfig`` (``/root/reference/appconfig.local.yaml:5-10``)."""

    hosts: List[str] = field(default_factory=list, metadata=_k("hosts", "list"))  # contact points
    port: int = field(default=9042, metadata=_k("port"))  # native protocol port
    user: str = field(default="", metadata=_k("user"))  # PasswordAuthenticator user; empty = no auth
    password: str = field(default="", metadata=_k("password", secret=True))  # PasswordAuthenticator password
    local_dc: str = field(default="", metadata=_k("local-dc"))  # DC-aware routing: prefer this DC's nodes
    # extensions
    keyspace: str = field(default="nexus", metadata=_k("keyspace"))  # keyspace of the checkpoints table
    table: str = field(default="checkpoints", metadata=_k("table"))  # checkpoints table (nexus-core schema)
    # consistency of reads and writes; conditional writes use the matching SERIAL level
    consistency: str = field(default="LOCAL_QUORUM", metadata=_k("consistency"))
    # connections per node when the node is not sharded (or shard-aware is off)
    connections_per_host: int = field(default=2, metadata=_k("connections-per-host"))
    request_timeout: float = field(default=5.0, metadata=_k("request-timeout", "duration"))  # per CQL request
    connect_timeout: float = field(default=5.0, metadata=_k("connect-timeout", "duration"))  # TCP + STARTUP
    # send each statement to a replica owning its partition token (ring from system.peers)
    token_aware: bool = field(default=True, metadata=_k("token-aware"))
    # Scylla shard-aware routing (scylladb/gocql fork, /root/reference/go.mod:93): one
    # connection per shard through the shard-aware port, requests to the owning shard
    shard_aware: bool = field(default=True, metadata=_k("shard-aware"))
    connections_per_shard: int = field(default=1, metadata=_k("connections-per-shard"))  # with shard-aware


@dataclass
class CompatConfig:
    """Switches for reference quirks; defaults keep observable parity
    where it is harmless and fix the hazards."""

    # "Algorithm encountered a fatal error during execution: Algorithm encountered ..."
    # (/root/reference/services/supervisor.go:198,325)
    doubled_fatal_cause: bool = field(default=True, metadata=_k("doubled-fatal-cause"))
    # full-row INSERT (reference) vs owned-columns UPDATE (this build's default)
    full_row_upsert: bool = field(default=False, metadata=_k("full-row-upsert"))
    # delete the Job when the checkpoint read fails (supervisor.go:265-273)
    delete_on_read_error: bool = field(default=False, metadata=_k("delete-on-read-error"))
    # NotFound on Job DELETE counts as success (fixes retry hazard)
    delete_not_found_ok: bool = field(default=True, metadata=_k("delete-not-found-ok"))
    # conditional writes (LWT ``IF lifecycle_stage IN (<unfinished stages>)``): a write never
    # moves a row out of a finished stage, so a deposed leader's queued decision cannot
    # overwrite what the new leader (or another component: CANCELLED) wrote.
    #   auto   — ToRunning always conditional; failure writes conditional when leader
    #            election is enabled (HA) — the default
    #   always — every write conditional; never — none (reference behaviour)
    # true / false are accepted as always / never.
    conditional_update: str = field(default="auto", metadata=_k("conditional-update"))
    # one store call per decision: the conditional write alone decides (its not-applied
    # answer carries the row's stage: no row / finished / already RUNNING) instead of the
    # reference's read followed by a write (supervisor.go:264-301).  That write is a
    # lightweight transaction — a Paxos round, ~4 replica round trips and serialised per
    # partition where a plain write takes 1 (docs/ARCHITECTURE.md "Pricing the LWT"):
    #   auto  — fused only under HA (leader election or shard leases: a deposed owner may
    #           still hold a decision), else the reference's read + plain write — default
    #   true  — always fused;  false — never (the reference's read + write)
    # Off with conditional-update: never or full-row-upsert.
    fused_write: str = field(default="auto", metadata=_k("fused-write"))


@dataclass
class CircuitBreakerConfig:
    """Circuit breaker in front of the checkpoint store (parallel/breaker.py): during a
    store outage decisions wait in the queue instead of burning their retries."""

    enabled: bool = field(default=True, metadata=_k("enabled"))
    # consecutive store failures that open the circuit
    failure_threshold: int = field(default=5, metadata=_k("failure-threshold"))
    # first open period; doubled on every re-open (failed probe) up to max-open-duration
    open_duration: float = field(default=1.0, metadata=_k("open-duration", "duration"))
    max_open_duration: float = field(default=30.0, metadata=_k("max-open-duration", "duration"))


@dataclass
class LabelConfig:
    """Label keys of nexus-core ``checkpoint/models`` (values unverified offline,
    SURVEY §8 q2) — configurable so a deployment can pin the real strings."""

    nexus_component_label: str = field(default="science.sneaksanddata.com/nexus-component", metadata=_k("nexus-component"))
    algorithm_run_value: str = field(default="algorithm-run", metadata=_k("algorithm-run-value"))
    job_template_name_key: str = field(default="science.sneaksanddata.com/algorithm-template-name", metadata=_k("job-template-name"))
    job_name_label: str = field(default="batch.kubernetes.io/job-name", metadata=_k("job-name"))


@dataclass
class RulesConfig:
    """Classifier extensions beyond the reference decision table (SURVEY §2.9.1 gaps)."""

    # also classify Event *updates* (repeat counts), not only adds (the reference: adds only)
    handle_event_updates: bool = field(default=True, metadata=_k("handle-event-updates"))
    # classify pod status (OOMKilled, HIP OOM, image pull, config errors, crash loops) beyond
    # the reference's event table
    pod_status_rules: bool = field(default=True, metadata=_k("pod-status-rules"))
    # Evicted pods: "fail" the run immediately, or "observe" (record evidence, let the
    # Job controller retry and enrich the terminal Job event)
    evicted_policy: str = field(default="observe", metadata=_k("evicted-policy"))
    # a pod its node's kubelet refused at admission (UnexpectedAdmissionError — the GPU device
    # plugin could not allocate —, OutOf<resource>, TopologyAffinityError, NodeAffinity…):
    # "fail" the run (SCHEDULING_FAILED, class gpu-admission / admission), or "observe"
    # (record it; the Job's BackoffLimitExceeded is then written with that cause)
    admission_policy: str = field(default="fail", metadata=_k("admission-policy"))
    # after a restart: runs whose pod is running but whose Started Event is not in the Event
    # list (it expired — the API server keeps Events ~1 h — while the supervisor was down)
    # get a ToRunning decision, at most this many per second and only while no decision is
    # queued (a backlog of failures is never delayed); 0 = off (the reference: never)
    running_sweep_rate: float = field(default=5.0, metadata=_k("running-sweep-rate", "number"))
    # wait this long after the caches synced before sweeping (the replayed Events decide first)
    running_sweep_delay: float = field(default=30.0, metadata=_k("running-sweep-delay", "duration"))
    # FailedScheduling (e.g. insufficient amd.com/gpu): fail after this long unschedulable; 0 = never
    unschedulable_timeout: float = field(default=0.0, metadata=_k("unschedulable-timeout", "duration"))
    # keep events whose involved object is not cached yet this long before dropping as stale
    stale_event_grace: float = field(default=2.0, metadata=_k("stale-event-grace", "duration"))
    # trace column format: raw (reference: event message), json, or auto (json when extra evidence exists)
    trace_format: str = field(default="auto", metadata=_k("trace-format"))
    # cap on the trace column's size (bytes of JSON); larger documents are trimmed
    # deterministically (least telling detail first); 0 = no cap
    trace_max_bytes: int = field(default=8192, metadata=_k("trace-max-bytes"))
    # a BackoffLimitExceeded Job decision whose pods died of an OOM or were evicted:
    # true — write FAILED with the OOM / eviction cause, the same row the pod-status OOM
    # rule and ``evicted-policy: fail`` write, so the stage does not depend on which
    # decision is applied first; false — keep the reference's DEADLINE_EXCEEDED for
    # BackoffLimitExceeded (supervisor.go:183-193), the class and evidence go into the
    # trace only (docs/PARITY.md)
    oom_fails_backoff_job: bool = field(default=True, metadata=_k("oom-fails-backoff-job"))
    # a Job's BackoffLimitExceeded / PodFailurePolicy says one of its pods failed, but Pods
    # and Jobs (and Events) arrive on separate watch streams: when no cached pod of the Job
    # shows that failure yet, wait this long for the pod's update before the decision is
    # written, so its cause (OOM, eviction, GPU) does not depend on stream order; 0 = off
    job_pod_settle: float = field(default=1.0, metadata=_k("job-pod-settle", "duration"))


@dataclass
class GpuConfig:
    """MI355X attribution (north star in BASELINE.json)."""

    # enrich failing GPU decisions with GPU evidence, RCCL/xGMI topology and the OOM verdict
    attribution_enabled: bool = field(default=True, metadata=_k("attribution-enabled"))
    hbm_capacity_gb: float = field(default=288.0, metadata=_k("hbm-capacity-gb"))  # per GPU (MI355X: 288)
    # a pod's own VRAM peak at or above this share of capacity, with a failed exit, is HBM OOM
    hbm_oom_fraction: float = field(default=0.97, metadata=_k("hbm-oom-fraction"))
    # pod annotation the node agent writes its GPU evidence to
    evidence_annotation: str = field(default="nexus.amd.com/gpu-evidence", metadata=_k("evidence-annotation"))
    # extended resource that marks a GPU pod
    gpu_resource_name: str = field(default="amd.com/gpu", metadata=_k("gpu-resource-name"))
    backend: str = field(default="auto", metadata=_k("backend"))  # auto | amdsmi | fake | none
    sample_interval: float = field(default=0.5, metadata=_k("sample-interval", "duration"))  # amd-smi VRAM sampling
    # read GPUs of the node this process runs on (in-node supervisor / bench); the cluster
    # deployment instead reads the node agents' pod annotations
    local_telemetry: bool = field(default=False, metadata=_k("local-telemetry"))
    # amd-smi event listener (VM faults, resets) next to the VRAM sampler; off = sampling only
    telemetry_events: bool = field(default=True, metadata=_k("telemetry-events"))
    # hold a failed GPU pod's decision this long for the node agent's evidence annotation
    # (0 = decide immediately on whatever is there)
    evidence_wait: float = field(default=0.0, metadata=_k("evidence-wait", "duration"))
    # container log tails for the OOM signature of a failed GPU container whose termination
    # message is empty (the default terminationMessagePolicy: File; torch prints its OOM to
    # stderr): auto — the node agent's /var/log/pods reading when its annotation has one,
    # else the supervisor GETs pods/<pod>/log (RBAC pods/log get); api — always the API;
    # node — the agent's reading only; off — never look at logs
    log_tail: str = field(default="auto", metadata=_k("log-tail"))
    # longest a decision waits for an outstanding log-tail fetch
    log_tail_timeout: float = field(default=2.0, metadata=_k("log-tail-timeout", "duration"))
    log_tail_bytes: int = field(default=65536, metadata=_k("log-tail-bytes"))  # limitBytes of a tail
    # pods/log reads in flight at once per process (proxied through the kubelet: the most
    # expensive read there is); a GPU failure wave queues behind this bound
    log_tail_concurrency: int = field(default=8, metadata=_k("log-tail-concurrency"))


@dataclass
class StagesConfig:
    """nexus-core ``models.LifecycleStage*`` strings and ``IsFinished()`` set (SURVEY §8 q1:
    only BUFFERED / RUNNING / CANCELLED are attested by the reference's seed data, the
    rest are unverifiable offline) — pinned per deployment."""

    new: str = field(default="NEW", metadata=_k("new"))
    buffered: str = field(default="BUFFERED", metadata=_k("buffered"))
    running: str = field(default="RUNNING", metadata=_k("running"))
    completed: str = field(default="COMPLETED", metadata=_k("completed"))
    failed: str = field(default="FAILED", metadata=_k("failed"))
    scheduling_failed: str = field(default="SCHEDULING_FAILED", metadata=_k("scheduling-failed"))
    deadline_exceeded: str = field(default="DEADLINE_EXCEEDED", metadata=_k("deadline-exceeded"))
    cancelled: str = field(default="CANCELLED", metadata=_k("cancelled"))
    # stage strings for which IsFinished() is true (may name stages this build does not model,
    # e.g. one added by a newer nexus-core); empty = the five terminal stages above
    finished: List[str] = field(default_factory=list, metadata=_k("finished", "list"))

    def mapping(self):
        return {"NEW": self.new, "BUFFERED": self.buffered, "RUNNING": self.running, "COMPLETED": self.completed,
                "FAILED": self.failed, "SCHEDULING_FAILED": self.scheduling_failed,
                "DEADLINE_EXCEEDED": self.deadline_exceeded, "CANCELLED": self.cancelled}

    def apply(self) -> None:
        """Make these the process-wide stage strings (models.checkpoint)."""
        from ..models.checkpoint import configure_lifecycle_stages

        configure_lifecycle_stages(self.mapping(), self.finished or None)


@dataclass
class LeaderElectionConfig:
    """Lease-based active/standby (``ha/leader.py``); the timings also drive shard leases."""

    # one active replica holds a coordination.k8s.io Lease; standbys keep warm caches
    enabled: bool = field(default=False, metadata=_k("enabled"))
    lease_name: str = field(default="nexus-supervisor-leader", metadata=_k("lease-name"))  # Lease object name
    # how long a Lease stays held without renewal before another replica may take it
    lease_duration: float = field(default=15.0, metadata=_k("lease-duration", "duration"))
    # the holder stops acting this long after its last successful renewal *started* (bounded
    # renewals + a watchdog), so a partitioned holder stops before anyone can take over
    renew_deadline: float = field(default=10.0, metadata=_k("renew-deadline", "duration"))
    retry_period: float = field(default=2.0, metadata=_k("retry-period", "duration"))  # renew / acquire interval
    identity: str = field(default="", metadata=_k("identity"))  # holder identity; empty = pod name


@dataclass
class ShardingConfig:
    """Hash sharding of runs across replicas (``parallel/sharding.py``; 1 shard = off).

    ``static``: this replica owns ``shard-index`` (StatefulSet ordinal).  ``lease``: one
    Lease per shard (``<leader-election.lease-name>-shard-<k>``, leader-election timings);
    each replica holds up to its fair share ``ceil(shards / replicas)`` and takes over any
    shard left unheld for a full lease duration, so shards fail over individually."""

    shards: int = field(default=1, metadata=_k("shards"))  # runs split into this many shards; 1 = off
    shard_index: int = field(default=0, metadata=_k("shard-index"))  # static mode: the shard this replica owns
    mode: str = field(default="static", metadata=_k("mode"))  # static | lease
    # expected replica count (Helm replicaCount) for the lease-mode fair share; 0 = greedy
    replicas: int = field(default=0, metadata=_k("replicas"))
    # label carrying a run's shard (shard_of(job name, shards), ``python -m
    # nexus_supervisor_amd shard-of``) on its Job and pod template, stamped by the component
    # that submits the Job: a replica then watches only its shards' Pods and Jobs
    # (``<label> in (owned…)``, filtered by the API server's watch cache) instead of every
    # replica receiving the whole namespace.  Events carry no such label and stay a full
    # stream (dropped before decode by the native router).  Empty = off.  Jobs without the
    # label are invisible with it on: /metrics shard_label_missing counts them and the audit
    # re-stamps them (audit-interval, repair-labels)
    shard_label: str = field(default="", metadata=_k("shard-label"))
    # serve the mutating admission webhook that stamps shard-label on Nexus Jobs (and their
    # pod templates) and Pods at CREATE (admission.py; the chart registers it with
    # failurePolicy: Ignore); 0 = off
    webhook_port: int = field(default=0, metadata=_k("webhook-port"))
    # tls.crt / tls.key of the webhook's serving certificate (a Secret mounted here; with
    # webhook-cert-bootstrap a writable directory the replica writes its pair to)
    webhook_cert_dir: str = field(default="/etc/nexus/webhook-tls", metadata=_k("webhook-cert-dir"))
    # no cert-manager: the replicas mint a self-signed CA + serving certificate into the
    # Secret webhook-secret (compare-and-swap: one pair for all), renew it 30 days before
    # expiry, and keep caBundle of webhook-config-name in step (webhook_certs.py)
    webhook_cert_bootstrap: bool = field(default=False, metadata=_k("webhook-cert-bootstrap"))
    webhook_secret: str = field(default="nexus-supervisor-webhook-tls", metadata=_k("webhook-secret"))
    # the MutatingWebhookConfiguration whose caBundle the bootstrap sets; empty = leave it alone
    webhook_config_name: str = field(default="", metadata=_k("webhook-config-name"))
    # the webhook Service's name (the certificate's DNS names: <service>.<namespace>.svc…)
    webhook_service: str = field(default="nexus-supervisor-webhook", metadata=_k("webhook-service"))
    # at startup (static mode) / on gaining a shard (lease mode): re-stamp the label of this
    # replica's runs whose label was computed for another shard count
    relabel: bool = field(default=True, metadata=_k("relabel"))
    # the shard-label audit: every interval, LIST the Nexus Jobs / Pods whose label is missing
    # or names no shard (shard_label_missing) — admitted while the webhook was unreachable
    # (failurePolicy: Ignore) and invisible to every replica; 0 = off
    audit_interval: float = field(default=60.0, metadata=_k("audit-interval", "duration"))
    # the audit PATCHes the label of the runs of this replica's shards it finds (self-healing:
    # a run submitted during a webhook outage is supervised within one audit interval);
    # false = count and log only
    repair_labels: bool = field(default=True, metadata=_k("repair-labels"))
    # every this many audit passes, also re-check the runs labelled with this replica's shards
    # and fix labels that disagree with shard_of(name, shards) (shard_label_wrong: a stale
    # count stamped during a rolling change of shards)
    relabel_every: int = field(default=5, metadata=_k("relabel-every"))


@dataclass
class RuntimeConfig:
    """Python runtime tuning for a large, long-lived informer cache (see ``utils/gctune.py``)."""

    # after the initial cache sync: collect once, then move every surviving object to the
    # permanent generation so full collections stop re-traversing 10k cached runs
    gc_freeze: bool = field(default=True, metadata=_k("gc-freeze"))
    gc_threshold0: int = field(default=200000, metadata=_k("gc-threshold0"))  # CPython default 700
    gc_threshold1: int = field(default=20, metadata=_k("gc-threshold1"))  # CPython default 10
    gc_threshold2: int = field(default=20, metadata=_k("gc-threshold2"))  # CPython default 10
    gc_refreeze_interval: float = field(default=600.0, metadata=_k("gc-refreeze-interval", "duration"))  # 0 = never
    # process-per-core runtime: this many shard-worker processes, each owning the runs whose
    # job name hashes to it (informers filter at ingest), under one coordinating parent that
    # holds the lease and serves /metrics; 1 = single-process supervisor; 0 = one per CPU of
    # the container's share (cgroup quota / affinity) minus one for the parent, at most 6
    worker_processes: int = field(default=1, metadata=_k("worker-processes"))
    # set by the coordinator in each worker process (not a user knob)
    worker_index: int = field(default=0, metadata=_k("worker-index"))
    # with worker processes: the parent holds one LIST+WATCH per kind and routes each object
    # to its owner worker (parallel/watchhub.py) instead of every worker watching everything
    watch_hub: bool = field(default=True, metadata=_k("watch-hub"))
    # CPU placement of the supervisor's processes (utils/affinity.py), set at start-up and
    # inherited by the shard workers: none = the scheduler's (or the pod cpuset's); numa =
    # the NUMA node of the host's first GPU (node 0 without one); numa-cores = that node,
    # one hardware thread per physical core; auto = numa-cores, else numa, when either
    # leaves at least worker-processes + 1 CPUs of the allowed set
    cpu_affinity: str = field(default="none", metadata=_k("cpu-affinity"))


@dataclass
class ObservabilityConfig:
    # DogStatsD metric namespace (the reference: nexus_receiver)
    statsd_name: str = field(default="nexus_supervisor", metadata=_k("statsd-name"))
    http_port: int = field(default=0, metadata=_k("http-port"))  # /metrics /healthz /readyz /debug/pprof; 0 = off
    http_host: str = field(default="0.0.0.0", metadata=_k("http-host"))  # bind address of the HTTP endpoints
    profiler_hz: int = field(default=97, metadata=_k("profiler-hz"))  # /debug/pprof sampling rate
    # per-decision stage timestamps -> stage_classify/queue/read/write/delete histograms
    stage_timestamps: bool = field(default=True, metadata=_k("stage-timestamps"))
    # a Kubernetes Warning Event (reason NexusRunFailed) on the Job per failing decision:
    # stage, failure class, GPU and cause in `kubectl describe job` (RBAC: events create)
    record_events: bool = field(default=False, metadata=_k("record-events"))


@dataclass
class SupervisorConfig:
    """``app.SupervisorConfig`` (``/root/reference/app/app_config.go:8-20``) + extensions."""

    astra_cql_store: AstraBundleConfig = field(default_factory=AstraBundleConfig, metadata=_k("astra-cql-store"))
    scylla_cql_store: ScyllaCqlStoreConfig = field(default_factory=ScyllaCqlStoreConfig, metadata=_k("scylla-cql-store"))
    cql_store_type: str = field(default=CQL_STORE_ASTRA, metadata=_k("cql-store-type"))  # astra | scylla | memory
    kube_config_path: str = field(default="", metadata=_k("kube-config-path"))  # empty = in-cluster service account
    resource_namespace: str = field(default="nexus", metadata=_k("resource-namespace"))  # namespace of the runs' Jobs
    log_level: str = field(default="INFO", metadata=_k("log-level"))  # DEBUG | INFO | WARN | ERROR
    # first retry backoff of a run
    failure_rate_base_delay: float = field(default=0.1, metadata=_k("failure-rate-base-delay", "duration"))
    failure_rate_max_delay: float = field(default=1.0, metadata=_k("failure-rate-max-delay", "duration"))  # backoff cap
    # token bucket; 0 = uncapped
    rate_limit_elements_per_second: float = field(default=10, metadata=_k("rate-limit-elements-per-second", "number"))
    rate_limit_elements_burst: int = field(default=100, metadata=_k("rate-limit-elements-burst"))  # bucket size
    workers: int = field(default=2, metadata=_k("workers"))  # concurrent decisions per replica
    # ---- extensions ----
    resync_period: float = field(default=30.0, metadata=_k("resync-period", "duration"))  # informer resync
    # server-side label selector on the Pod/Job informers (only Nexus runs are cached)
    informer_label_selector: bool = field(default=True, metadata=_k("informer-label-selector"))
    # server-side field selector on the Event informer: reason!=<each Normal start/stop reason
    # no rule reads> (Scheduled, Pulling, Pulled, Created, Killing, SuccessfulCreate, ...)
    informer_event_noise_selector: bool = field(default=True, metadata=_k("informer-event-noise-selector"))
    watch_timeout: float = field(default=300.0, metadata=_k("watch-timeout", "duration"))  # server-side watch timeout
    # client-side API flow control (client-go rest.Config QPS / Burst): a token bucket in
    # front of every API request of a replica (Job DELETEs, pods/log reads, Events, LIST /
    # WATCH; Lease calls exempt), divided over its shard-worker processes.  The reference
    # runs on client-go's defaults, 5 / 10 (app_dependencies.go:39-45) — that holds a
    # 1,000-pod failure wave's DELETEs for 200 s; 50 / 100 is a controller-class client.
    # 0 = no client-side limit (the server's API Priority and Fairness still answers 429)
    kube_qps: float = field(default=50.0, metadata=_k("kube-qps", "number"))
    kube_burst: int = field(default=100, metadata=_k("kube-burst"))
    # 429 (and 5xx with Retry-After) answers re-sent after the server's Retry-After, at most
    # this many times per request (client-go: 10); 0 = never
    kube_max_retries: int = field(default=10, metadata=_k("kube-max-retries"))
    max_retries: int = field(default=16, metadata=_k("max-retries"))  # 0 = retry forever
    # issue the Job DELETE after the checkpoint write without holding a worker (retried
    # in the background with the failure backoff); false = delete inside the worker
    async_job_delete: bool = field(default=True, metadata=_k("async-job-delete"))
    # shadow mode for a migration: classify and decide as usual, read checkpoints, but never
    # write a row or delete a Job — each would-be action is logged and counted (dry_run_*)
    dry_run: bool = field(default=False, metadata=_k("dry-run"))
    compat: CompatConfig = field(default_factory=CompatConfig, metadata=_k("compat"))
    circuit_breaker: CircuitBreakerConfig = field(default_factory=CircuitBreakerConfig, metadata=_k("circuit-breaker"))
    labels: LabelConfig = field(default_factory=LabelConfig, metadata=_k("labels"))
    stages: StagesConfig = field(default_factory=StagesConfig, metadata=_k("stages"))
    rules: RulesConfig = field(default_factory=RulesConfig, metadata=_k("rules"))
    gpu: GpuConfig = field(default_factory=GpuConfig, metadata=_k("gpu"))
    leader_election: LeaderElectionConfig = field(default_factory=LeaderElectionConfig, metadata=_k("leader-election"))
    sharding: ShardingConfig = field(default_factory=ShardingConfig, metadata=_k("sharding"))
    observability: ObservabilityConfig = field(default_factory=ObservabilityConfig, metadata=_k("observability"))
    runtime: RuntimeConfig = field(default_factory=RuntimeConfig, metadata=_k("runtime"))


class ConfigError(ValueError):
    pass


def validate(cfg: SupervisorConfig) -> SupervisorConfig:
    if cfg.cql_store_type not in CQL_STORE_TYPES:
        raise ConfigError(f"unknown store type {cfg.cql_store_type}")
    from ..obs.logging import parse_level

    try:
        parse_level(cfg.log_level)
    except ValueError as exc:
        raise ConfigError(str(exc)) from None
    if cfg.workers < 1:
        raise ConfigError(f"workers must be >= 1, got {cfg.workers}")
    if cfg.rate_limit_elements_per_second < 0:
        raise ConfigError("rate-limit-elements-per-second must be >= 0 (0 = unlimited)")
    if cfg.rate_limit_elements_burst < 1:
        raise ConfigError("rate-limit-elements-burst must be >= 1")
    if cfg.failure_rate_base_delay < 0 or cfg.failure_rate_max_delay < cfg.failure_rate_base_delay:
        raise ConfigError("failure-rate-max-delay must be >= failure-rate-base-delay >= 0")
    cu = str(cfg.compat.conditional_update).strip().lower()
    cfg.compat.conditional_update = {"true": "always", "1": "always", "yes": "always", "on": "always",
                                     "false": "never", "0": "never", "no": "never", "off": "never"}.get(cu, cu)
    if cfg.compat.conditional_update not in ("auto", "always", "never"):
        raise ConfigError("compat.conditional-update must be auto|always|never")
    fw = str(cfg.compat.fused_write).strip().lower()
    cfg.compat.fused_write = {"1": "true", "yes": "true", "on": "true", "always": "true",
                              "0": "false", "no": "false", "off": "false", "never": "false"}.get(fw, fw)
    if cfg.compat.fused_write not in ("auto", "true", "false"):
        raise ConfigError("compat.fused-write must be auto|true|false")
    st = cfg.stages.mapping()
    if any(not v for v in st.values()) or len(set(st.values())) != len(st):
        raise ConfigError("stages: every lifecycle stage needs a distinct non-empty string")
    if set(cfg.stages.finished) & {st["NEW"], st["BUFFERED"], st["RUNNING"]}:
        raise ConfigError("stages.finished cannot contain new / buffered / running")
    if cfg.rules.evicted_policy not in ("fail", "observe"):
        raise ConfigError("rules.evicted-policy must be fail|observe")
    if cfg.rules.running_sweep_rate < 0 or cfg.rules.running_sweep_delay < 0:
        raise ConfigError("rules.running-sweep-rate and rules.running-sweep-delay must be >= 0")
    if cfg.rules.admission_policy not in ("fail", "observe"):
        raise ConfigError("rules.admission-policy must be fail|observe")
    if cfg.rules.trace_format not in ("raw", "json", "auto"):
        raise ConfigError("rules.trace-format must be raw|json|auto")
    if cfg.rules.trace_max_bytes and cfg.rules.trace_max_bytes < 1024:
        raise ConfigError("rules.trace-max-bytes must be 0 (no cap) or >= 1024")
    if cfg.sharding.shards < 1 or not 0 <= cfg.sharding.shard_index < cfg.sharding.shards:
        raise ConfigError("sharding.shard-index must be in [0, shards)")
    if cfg.sharding.mode not in ("static", "lease"):
        raise ConfigError("sharding.mode must be static|lease")
    if cfg.sharding.replicas < 0:
        raise ConfigError("sharding.replicas must be >= 0 (0 = greedy)")
    if cfg.sharding.audit_interval < 0 or cfg.sharding.relabel_every < 1:
        raise ConfigError("sharding.audit-interval must be >= 0 (0 = off) and sharding.relabel-every >= 1")
    rt = cfg.runtime
    if rt.worker_processes == 0:
        from ..utils.cpus import auto_worker_processes

        rt.worker_processes = auto_worker_processes()
    if rt.worker_processes < 1 or not 0 <= rt.worker_index < rt.worker_processes:
        raise ConfigError("runtime.worker-processes must be >= 0 (0 = auto) and runtime.worker-index in [0, worker-processes)")
    if rt.cpu_affinity not in ("none", "numa", "numa-cores", "auto"):
        raise ConfigError("runtime.cpu-affinity must be none|numa|numa-cores|auto")
    if not 0 < cfg.gpu.hbm_oom_fraction <= 1:
        raise ConfigError("gpu.hbm-oom-fraction must be in (0, 1]")
    if cfg.gpu.log_tail not in ("auto", "api", "node", "off"):
        raise ConfigError("gpu.log-tail must be auto|api|node|off")
    if cfg.gpu.log_tail_bytes < 1024 or cfg.gpu.log_tail_timeout <= 0:
        raise ConfigError("gpu.log-tail-bytes must be >= 1024 and gpu.log-tail-timeout > 0")
    if cfg.gpu.log_tail_concurrency < 1:
        raise ConfigError("gpu.log-tail-concurrency must be >= 1")
    if cfg.kube_qps < 0 or cfg.kube_burst < 1 or cfg.kube_max_retries < 0:
        raise ConfigError("kube-qps must be >= 0 (0 = no limit), kube-burst >= 1, kube-max-retries >= 0")
    if cfg.leader_election.enabled or cfg.sharding.mode == "lease":
        le = cfg.leader_election
        if not le.lease_duration > le.renew_deadline > le.retry_period > 0:
            raise ConfigError("leader-election: lease-duration > renew-deadline > retry-period > 0 required")
    return cfg
