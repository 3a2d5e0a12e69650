"""Workload models run inside pool pods (validation jobs)."""
