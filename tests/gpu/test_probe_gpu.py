"""Real-MI355X tests of the gfx950 HIP probe kernels (run on the GPU box with ``-m gpu``).

Numerics: the MFMA GEMM is checked bit-exactly against an fp32 VALU reference (256^3, asymmetric
operands) and exact ABFT row/column checksums (N^3, modulo 2^32); the HBM test compares every bit. These tests also
prove the checkers *detect* corruption by injecting faults between compute and check.
"""
from __future__ import annotations

import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NATIVE = os.path.join(ROOT, "build", "native")


@pytest.fixture(scope="module")
def hip(native_built):
    from gpupool.ops import probe
    n = probe.init()
    assert n >= 1, "no HIP device visible"
    return probe


def test_mfma_fragment_layout_selftest(native_built):
    r = subprocess.run([os.path.join(NATIVE, "probe_selftest")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout)
    assert out["mfma_layout_mismatches"] == 0 and out["mfma16_layout_mismatches"] == 0


def test_identify_is_gfx950(hip):
    info = hip.identify(0)
    assert info["gcnArch"].startswith("gfx950")
    assert info["hipUUID"].startswith("GPU-")
    assert info["computeUnits"] == 256


def test_probe_passes_and_is_fast(hip):
    r = hip.run(0, hbm_bytes=1 << 30)
    assert r["passed"], r
    assert r["hbm"]["badBits"] == 0 and r["mfma"]["elementMismatches"] == 0
    assert r["mfma"]["abftMismatches"] == 0
    # sanity floors well below what MI355X reaches (~5 TB/s, ~750 TF): catch a broken kernel
    assert r["hbm"]["GBps"] > 2000, r["hbm"]
    assert r["mfma"]["tflops"] > 300, r["mfma"]
    assert r["ms"] < 1000


def test_hbm_checker_counts_injected_bit_flips(hip):
    r = hip.run(0, hbm_bytes=256 << 20, mfma=False, injectBitFlips=37)
    assert not r["passed"]
    assert r["hbm"]["badBits"] == 37  # every flipped bit found, nothing else
    assert r["hbm"]["firstBadOffset"] is not None


def test_abft_detects_single_corrupted_element(hip):
    r = hip.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=1024, injectGemmFault=1)
    assert not r["passed"]
    assert r["mfma"]["abftMismatches"] == 2  # its row and its column checksum
    assert r["mfma"]["elementMismatches"] == 0


def test_probe_cli(native_built):
    r = subprocess.run([os.path.join(NATIVE, "mi355x-probe"), "--hbm-bytes", str(64 << 20),
                        "--gemm-n", "1024"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for line in r.stdout.strip().splitlines():
        assert json.loads(line)["passed"]


@pytest.mark.parametrize("n", [256, 512, 1280, 2048])
@pytest.mark.parametrize("tile", [128, 256])
def test_gemm_kernels_exact_at_sizes(hip, n, tile):
    """Both GEMM kernels (256x256 glds and 128x128 register-staged) are bit-exact (ABFT) at
    several N, including one that is not a power of two (1280 = 5 x 256)."""
    r = hip.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=n, gemm_tile=tile)
    assert r["passed"], r
    assert r["mfma"]["tile"] == tile and r["mfma"]["n"] == n
    assert r["mfma"]["abftMismatches"] == 0 and r["mfma"]["elementMismatches"] == 0


def test_overlapped_and_serial_probe_agree(hip):
    """The two-stream probe (HBM test beside the MFMA phase) finds the same injected faults as
    the serial one and both pass clean runs."""
    for overlap in (0, 1):
        clean = hip.run(0, hbm_bytes=256 << 20, overlap=overlap)
        assert clean["passed"], clean
        bad = hip.run(0, hbm_bytes=256 << 20, gemm_n=1024, overlap=overlap, injectBitFlips=5,
                      injectGemmFault=1)
        assert not bad["passed"]
        assert bad["hbm"]["badBits"] == 5 and bad["mfma"]["abftMismatches"] == 2


def test_peer_copy_path(hip):
    """The xGMI peer check's copy + bit-exact verify path. On a 1-GPU box src == dst exercises
    it as a local device copy; with more GPUs visible, 0 -> 1 goes over an xGMI link."""
    n = hip.init()
    r = hip.peer(0, 0, 64 << 20)
    assert r["passed"] and r["canAccessPeer"] and r["badBits"] == 0, r
    assert r["GBps"] > 100, r
    if n > 1:
        x = hip.peer(0, 1, 64 << 20)
        assert x["passed"] and x["badBits"] == 0, x
        assert x["GBps"] > 10, x


def test_probe_arena_reused_then_trimmed(hip):
    """The ~1.2 GiB probe arena is kept between back-to-back probes (no hipMalloc on the claim
    path) and handed back by trim(); a probe after a trim allocates again and still passes."""
    hip.trim(0)
    a = hip.run(0, hbm_bytes=1 << 30)
    b = hip.run(0, hbm_bytes=1 << 30)
    assert a["passed"] and b["passed"]
    assert a["phases"]["arenaReused"] is False and b["phases"]["arenaReused"] is True
    assert b["phases"]["allocMs"] < a["phases"]["allocMs"]
    assert hip.trim(0) == 1 and hip.trim(0) == 0
    c = hip.run(0, hbm_bytes=1 << 30)
    assert c["passed"] and c["phases"]["arenaReused"] is False
    hip.trim(0)
