"""High availability: Lease leader election and run sharding."""
