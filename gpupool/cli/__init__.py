"""Command-line tools (gpuctl)."""
