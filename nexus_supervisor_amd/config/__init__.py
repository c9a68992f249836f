"""Configuration: typed schema + layered loader (defaults < YAML < env overlay < NEXUS__ env)."""
from .loader import ENV_PREFIX, env_name, from_mapping, iter_keys, load_config, redacted, to_mapping
from .schema import (
    CQL_STORE_ASTRA,
    CQL_STORE_MEMORY,
    CQL_STORE_SCYLLA,
    AstraBundleConfig,
    CompatConfig,
    ConfigError,
    GpuConfig,
    LabelConfig,
    LeaderElectionConfig,
    ObservabilityConfig,
    RulesConfig,
    ScyllaCqlStoreConfig,
    ShardingConfig,
    SupervisorConfig,
    validate,
)

__all__ = [
    "ENV_PREFIX", "env_name", "from_mapping", "iter_keys", "load_config", "redacted", "to_mapping",
    "CQL_STORE_ASTRA", "CQL_STORE_MEMORY", "CQL_STORE_SCYLLA",
    "AstraBundleConfig", "CompatConfig", "ConfigError", "GpuConfig", "LabelConfig",
    "LeaderElectionConfig", "ObservabilityConfig", "RulesConfig", "ScyllaCqlStoreConfig",
    "ShardingConfig", "SupervisorConfig", "validate",
]
