"""The in-repo AMD GPU operator: device plugin, labeller, exporter, partition manager, validator."""
