"""Shared utilities: KFD sysfs topology, configuration, Prometheus text format, logging."""
