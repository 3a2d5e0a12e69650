"""Native layer: C++ unit tests (plain, ASan+UBSan, TSan builds), C++/Python validation parity,
generated-artefact freshness (CRDs, constants header, protobuf descriptors)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from gpupool.apiserver_sim.store import ApiError, Store
from tests.conftest import make_native

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_cpp_unit_tests(native_built):
    r = subprocess.run([os.path.join(native_built, "gpupool_tests")], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " 0 failed" in r.stdout


@pytest.mark.slow
@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_cpp_unit_tests_under_sanitizers(san):
    """SURVEY.md §5 race-detection row: host code under ASan+UBSan and TSan."""
    r = make_native("host", san, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    exe = os.path.join(ROOT, "build", f"native-{san}", "gpupool_tests")
    r = subprocess.run([exe], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-6000:]


CASES = [
    {"kind": "Mi355xPool", "spec": {"replicas": 0}},
    {"kind": "Mi355xPool", "spec": {"replicas": 8, "resourceName": "amd.com/gpu-team-a"}},
    {"kind": "Mi355xPool", "spec": {"replicas": -1}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2000}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "resourceName": "Bad Name"}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "topologyPolicy": "ring"}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "health": {"thermal": "hot"}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "health": {"minXGMILinksUp": 9}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "probe": {"hbmBytes": 1024}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "probe": {"minMfmaTflops": 1000.5,
                                                             "minHbmGBps": 4000}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "probe": {"minMfmaTflops": -1}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2, "probe": {"xgmiPeerCheck": True,
                                                             "minXgmiGBps": 40,
                                                             "recheckSeconds": 300}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2, "probe": {"xgmiPeerCheck": "yes"}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2, "probe": {"recheckSeconds": -5}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "probe": {"minHbmGBps": "fast"}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "partition": {"compute": "CPX", "memory": "NPS4"}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "partition": {"compute": "XPX"}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "replacePolicy": "Never"}},
    {"kind": "Mi355xPool", "spec": {"replicas": 0, "autoscale": {"enabled": True, "maxReplicas": 4,
                                                                 "scaleDownDelaySeconds": 5}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 0, "autoscale": {"maxReplicas": 2000}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 0, "autoscale": {"minReplicas": -1}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 0, "autoscale": {"scaleDownDelaySeconds": -3}}},
    {"kind": "Mi355xPool", "spec": {}},
    {"kind": "Mi355xPool", "spec": {"replicas": 12, "maxNodes": 2}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "maxNodes": 0}},
    {"kind": "Mi355xPool", "spec": {"replicas": 1, "maxNodes": 65}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2, "sharing": {"replicasPerGPU": 4}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2, "sharing": {"replicasPerGPU": 0}}},
    {"kind": "Mi355xPool", "spec": {"replicas": 2, "sharing": {"replicasPerGPU": 65}}},
    {"kind": "AzureVmPool", "spec": {"replicas": 0, "resourceGroupName": "rg", "location": "e",
                                     "vmSize": "s", "vnetName": "v", "subnetName": "s",
                                     "azureCredentialSecret": "c",
                                     "imageReference": {"publisher": "p", "offer": "o", "sku": "s",
                                                        "version": "v"}}},
    {"kind": "AzureVmPool", "spec": {"replicas": -3, "resourceGroupName": "rg", "location": "e",
                                     "vmSize": "s", "vnetName": "v", "subnetName": "s",
                                     "azureCredentialSecret": "c",
                                     "imageReference": {"publisher": "p", "offer": "o", "sku": "s",
                                                        "version": "v"}}},
    {"kind": "AzureVmPool", "spec": {"replicas": 1, "resourceGroupName": "rg"}},
    {"kind": "Mi355xJob", "spec": {"replicas": 2, "template": {"spec": {}}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 4, "gpusPerReplica": 8, "poolRef": "p",
                                   "restartPolicy": "Never", "cleanPodPolicy": "All",
                                   "successPolicy": "Rank0", "ttlSecondsAfterFinished": 0,
                                   "template": {"spec": {"containers": [{"name": "m"}]}}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 0, "template": {}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1, "gpusPerReplica": 65, "template": {}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1, "restartPolicy": "Always", "template": {}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1, "masterPort": 0, "template": {}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1, "ttlSecondsAfterFinished": -2, "template": {}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1, "resourceName": "Bad", "template": {}}},
    {"kind": "Mi355xJob", "spec": {"replicas": 1, "cleanPodPolicy": "Some", "template": {}}},
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: json.dumps(c["spec"])[:60])
def test_validation_parity_cpp_vs_crd(case, tmp_path, native_built):
    """The manager's defensive validation agrees with the CRD OpenAPI admission."""
    import glob

    import yaml
    store = Store()
    crd_rt = store.types[("apiextensions.k8s.io", "customresourcedefinitions")]
    for p in glob.glob(os.path.join(ROOT, "config", "crd", "*.yaml")):
        store.create(crd_rt, None, yaml.safe_load(open(p)))
    plural = {"Mi355xPool": "mi355xpools", "AzureVmPool": "azurevmpools",
              "Mi355xJob": "mi355xjobs"}[case["kind"]]
    obj = {"apiVersion": "compute.my.domain/v1alpha1", "kind": case["kind"],
           "metadata": {"name": "x"}, "spec": case["spec"]}
    try:
        store.create(store.lookup("compute.my.domain", plural), "default", obj)
        py_ok = True
    except ApiError:
        py_ok = False
    f = tmp_path / "obj.json"
    f.write_text(json.dumps(obj))
    r = subprocess.run([os.path.join(native_built, "gpupool-manager"), "--validate", str(f)],
                       capture_output=True, text=True, timeout=30)
    cpp_ok = r.returncode == 0
    assert py_ok == cpp_ok, (py_ok, r.stdout)


def test_generated_manifests_are_fresh():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gen_manifests.py"),
                        "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_protobuf_descriptors_are_fresh():
    from gpupool.agent.deviceplugin import proto
    assert proto.regenerate(check=True)


def test_fake_fixture_is_fresh(tmp_path):
    """tests/fixtures/node_8x_mi355x{,_cpx}.json match their generator."""
    fxs = [os.path.join(ROOT, "tests", "fixtures", n)
           for n in ("node_8x_mi355x.json", "node_8x_mi355x_cpx.json")]
    before = [open(fx).read() for fx in fxs]
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "gen_fake_fixture.py")],
                   check=True, capture_output=True)
    assert [open(fx).read() for fx in fxs] == before


def test_share_library_needs_only_old_glibc(native_built):
    """libgpupool_share.so is loaded into arbitrary pod images through HSA_TOOLS_LIB, and ROCr
    skips a tools library that fails to load (the slot's limits would silently vanish). So it may
    need nothing but libc, at symbol versions every supported distro has (<= GLIBC_2.17), and may
    export only its three entry points (no std:: instantiations to interpose on the pod's own)."""
    import re
    lib = os.path.join(native_built, "libgpupool_share.so")
    dyn = subprocess.run(["objdump", "-p", lib], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"NEEDED\s+(\S+)", dyn)
    assert set(needed) <= {"libc.so.6"}, needed
    syms = subprocess.run(["objdump", "-T", lib], capture_output=True, text=True, check=True).stdout
    versions = set(re.findall(r"\((GLIBC[A-Z]*_[0-9.]+)\)", syms))
    assert not any(v.startswith("GLIBCXX") or v.startswith("CXXABI") for v in versions), versions
    newest = max(tuple(int(x) for x in v.split("_")[1].split(".")) for v in versions)
    assert newest <= (2, 17), versions
    exported = {ln.split()[-1] for ln in syms.splitlines() if " DF .text" in ln}
    assert exported == {"OnLoad", "OnUnload", "gpupool_share_stats"}, exported
