"""BASELINE config 1: AzureVmPool on the apiserver-sim with the FakeCloud provider (no cloud, no
GPU) — plus the reference guide's full contract (README.md:170-240): credentials Secret, tag-scoped
VMs, scale up/down, full cleanup of NIC + OS disk, finalizer-guarded delete."""
from __future__ import annotations

import json
import os
import time

import pytest
import yaml

from gpupool.kube import AZUREVMPOOLS, SECRETS

from .helpers import cond_is, conds, settled_events

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sample(name="gpu-pool-prod", replicas=2):
    doc = yaml.safe_load(open(os.path.join(ROOT, "config", "samples",
                                           "compute_v1alpha1_azurevmpool.yaml")))
    doc["metadata"]["name"] = name
    doc["spec"]["replicas"] = replicas
    return doc


def secret():
    return yaml.safe_load(open(os.path.join(ROOT, "config", "samples",
                                            "azure-credentials-secret.yaml")))


def az_ready(r):
    def pred(o):
        st = (o or {}).get("status") or {}
        return bool(o) and st.get("observedGeneration") == o["metadata"]["generation"] and \
            st.get("readyReplicas") == r and len(st.get("vms", [])) == r and \
            conds(o).get("Ready", {}).get("status") == "True"
    return pred


@pytest.fixture
def azure(cluster_factory, tmp_path):
    state = str(tmp_path / "cloud.json")
    c = cluster_factory(nodes=[], kinds="azure",
                        manager_args=["--fakecloud-state", state, "--credentials-retry", "300ms"])
    c.cloud_state = state
    return c


def cloud(c):
    return json.load(open(c.cloud_state))


def test_config1_replicas_zero_ready(azure):
    k = azure.client
    k.create(SECRETS, secret(), "default")
    k.create(AZUREVMPOOLS, sample("gpu-pool-zero", 0), "default")
    o = k.wait_for(AZUREVMPOOLS, "gpu-pool-zero", "default", az_ready(0), timeout=20)
    assert o["status"]["readyReplicas"] == 0
    assert "compute.my.domain/device-release" in o["metadata"]["finalizers"]
    assert conds(o)["CredentialsValid"]["status"] == "True"


def test_scale_up_down_and_cleanup(azure):
    k = azure.client
    k.create(SECRETS, secret(), "default")
    k.create(AZUREVMPOOLS, sample(replicas=2), "default")
    o = k.wait_for(AZUREVMPOOLS, "gpu-pool-prod", "default", az_ready(2), timeout=20)
    vms = cloud(azure)["vms"]
    assert len(vms) == 2
    assert all(v["tags"] == {"managed-by": "azurevmpool-operator", "owner": "default/gpu-pool-prod"}
               for v in vms)  # README.md:238 tag contract
    assert sorted(o["status"]["vms"]) == sorted(v["name"] for v in vms)
    k.patch(AZUREVMPOOLS, "gpu-pool-prod", {"spec": {"replicas": 1}}, "default")
    k.wait_for(AZUREVMPOOLS, "gpu-pool-prod", "default", az_ready(1), timeout=20)
    k.delete(AZUREVMPOOLS, "gpu-pool-prod", "default")
    k.wait_for(AZUREVMPOOLS, "gpu-pool-prod", "default", lambda o: o is None, timeout=20)
    st = cloud(azure)
    assert st["vms"] == []  # VM + NIC + OS disk all gone (README.md:216, :239)
    # the event recorder posts asynchronously (aggregated, off the reconcile path): wait for it
    deadline = time.monotonic() + 10
    while True:
        reasons = {e["reason"] for e in settled_events(k)}
        if {"VMCreating", "VMDeleting", "Finalized"} <= reasons or time.monotonic() > deadline:
            break
        time.sleep(0.05)
    assert {"VMCreating", "VMDeleting", "Finalized"} <= reasons


def test_missing_credentials_condition(azure):
    k = azure.client
    k.create(AZUREVMPOOLS, sample("nocreds", 1), "default")
    o = k.wait_for(AZUREVMPOOLS, "nocreds", "default",
                   cond_is("CredentialsValid", "False", "CredentialsMissing"), timeout=20)
    assert conds(o)["Ready"]["status"] == "False"
    k.create(SECRETS, secret(), "default")  # fixing the secret recovers without user action
    k.wait_for(AZUREVMPOOLS, "nocreds", "default", az_ready(1), timeout=20)


def test_async_provisioning_progressing(cluster_factory, tmp_path):
    c = cluster_factory(nodes=[], kinds="azure",
                        manager_args=["--fakecloud-provision-ms", "400"])
    k = c.client
    k.create(SECRETS, secret(), "default")
    k.create(AZUREVMPOOLS, sample("slow", 2), "default")
    o = k.wait_for(AZUREVMPOOLS, "slow", "default",
                   cond_is("Progressing", "True"), timeout=10)
    assert o["status"]["readyReplicas"] == 0 and len(o["status"]["vms"]) == 2
    k.wait_for(AZUREVMPOOLS, "slow", "default", az_ready(2), timeout=20)


def test_invalid_spec_rejected_at_admission(azure):
    from gpupool.kube import KubeError
    doc = sample("bad", -1)
    with pytest.raises(KubeError) as e:
        azure.client.create(AZUREVMPOOLS, doc, "default")
    assert e.value.code == 422 and "spec.replicas" in str(e.value)


def test_workload_identity_credentials(cluster_factory, tmp_path):
    """README.md:311 roadmap: Workload Identity instead of a static Secret. The manager's own
    federated identity (env + projected token file) is used when the pool names the
    'workload-identity' credential source."""
    token = tmp_path / "azure-identity-token"
    token.write_text("eyJhbGciOiJSUzI1NiJ9.fake.jwt\n")
    env = {"AZURE_CLIENT_ID": "11111111-2222-3333-4444-555555555555",
           "AZURE_TENANT_ID": "tenant", "AZURE_SUBSCRIPTION_ID": "sub",
           "AZURE_FEDERATED_TOKEN_FILE": str(token)}
    c = cluster_factory(nodes=[], kinds="azure", env=env,
                        manager_args=["--fakecloud-state", str(tmp_path / "cloud.json"),
                                      "--credentials-retry", "300ms"])
    k = c.client
    pool = sample("wi-pool", 1)
    pool["spec"]["azureCredentialSecret"] = "workload-identity"
    k.create(AZUREVMPOOLS, pool, "default")  # note: no Secret exists
    o = k.wait_for(AZUREVMPOOLS, "wi-pool", "default", az_ready(1), timeout=20)
    assert conds(o)["CredentialsValid"]["reason"] == "WorkloadIdentity"
    # an empty projected token makes the credentials invalid (and the pool says why)
    token.write_text("")
    k.patch(AZUREVMPOOLS, "wi-pool", {"spec": {"replicas": 2}}, "default")
    o = k.wait_for(AZUREVMPOOLS, "wi-pool", "default",
                   cond_is("CredentialsValid", "False", "CredentialsMissing"), timeout=20)
    assert "federated token file" in conds(o)["CredentialsValid"]["message"]
