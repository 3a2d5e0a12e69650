"""Apiserver credentials rotate under a running manager + agent (tests/integration/rotation.py)."""
from __future__ import annotations

import pytest

from .rotation import run_rotation

pytestmark = pytest.mark.slow


def test_two_token_rotations_without_a_failed_reconcile(cluster_factory, tmp_path):
    r = run_rotation(cluster_factory, tmp_path)
    assert r["errors"] == 0, r["reconcile_lines"]
    assert r["reloads"] >= 2, r
    assert r["heartbeat_failures"] == 0 and r["heartbeats"] > 5, r
    assert r["auth_401s"] > 0, r  # the old tokens really were refused (and recovered from)
    assert r["agent_ready"] == "True"
