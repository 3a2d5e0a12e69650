"""CEL rules of the CRDs (``x-kubernetes-validations``) and the interpreter apiserver-sim runs them
with (gpupool/api/cel.py): a kube-apiserver rejects these specs at admission; so does the sim."""
from __future__ import annotations

import pytest

from gpupool.api import cel, schema
from gpupool.apiserver_sim.store import ApiError, Store


@pytest.mark.parametrize("src,self_,want", [
    ("1 + 2 * 3 == 7", None, True),
    ("7 / 2 == 3 && -7 / 2 == -3 && -7 % 2 == -1", None, True),  # truncating integer division
    ("has(self.a) ? self.a.b : false", {"a": {"b": True}}, True),
    ("has(self.a) ? self.a.b : false", {}, False),
    ("'x' in self.l && !('y' in self.l)", {"l": ["x"]}, True),
    ("self.missing == 1 || true", {}, True),     # an error on one side of || is absorbed
    ("true || self.missing == 1", {}, True),
    ("size(self.s) == 3 && size(self.l) == 0", {"s": "abc", "l": []}, True),
    ("self.x >= 1.5", {"x": 2}, True),
    ("!(1 < 2)", None, False),
    ("self.a.b.c == 'z'", {"a": {"b": {"c": "z"}}}, True),
])
def test_interpreter(src, self_, want):
    assert cel.evaluate(src, self_) is want


@pytest.mark.parametrize("src,self_", [
    ("self.missing == 1", {}),                     # a missing field is an error, not false
    ("self.missing == 1 && true", {}),
    ("1 / 0 == 0", None),
    ("'a' < 1", None),
])
def test_errors(src, self_):
    with pytest.raises(cel.CelError):
        cel.evaluate(src, self_)


def test_parse_errors():
    for bad in ("self.", "has(1)", "foo(self)", "1 +", "(1"):
        with pytest.raises(cel.CelError):
            cel.compile_rule(bad)


def _store():
    st = Store()
    crds = st.lookup("apiextensions.k8s.io", "customresourcedefinitions")
    for c in schema.all_crds():
        st.create(crds, None, c)
    return st, {t.kind: t for t in st.types.values()}


def test_crd_rules_reject_at_admission():
    st, kinds = _store()
    pools = kinds["Mi355xPool"]

    def pool(name, **spec):
        return st.create(pools, "default", {"apiVersion": pools.api_version, "kind": "Mi355xPool",
                                            "metadata": {"name": name},
                                            "spec": {"replicas": 1, **spec}})
    pool("ok")
    pool("slots", sharing={"replicasPerGPU": 4, "cuPerSlot": 64})
    pool("cpx", sharing={"replicasPerGPU": 4, "cuPerSlot": 2}, partition={"compute": "CPX"})
    for spec, msg in (({"sharing": {"replicasPerGPU": 4, "cuPerSlot": 128}}, "256 CUs"),
                      ({"sharing": {"replicasPerGPU": 2, "cuPerSlot": 4}}, "one CU per XCD"),
                      ({"autoscale": {"minReplicas": 5, "maxReplicas": 2}}, "must not exceed")):
        with pytest.raises(ApiError) as ei:
            pool("bad", **spec)
        assert ei.value.code == 422 and msg in str(ei.value)
    # an update is validated too
    with pytest.raises(ApiError):
        st.patch(pools, "default", "ok", {"spec": {"autoscale": {"minReplicas": 9,
                                                                 "maxReplicas": 1}}}, "merge")
    jobs = kinds["Mi355xJob"]
    with pytest.raises(ApiError) as ei:
        st.create(jobs, "default", {"apiVersion": jobs.api_version, "kind": "Mi355xJob",
                                    "metadata": {"name": "j"},
                                    "spec": {"replicas": 2, "minAvailable": 3, "template": {
                                        "spec": {"containers": [{"name": "c"}]}}}})
    assert "minAvailable must not exceed replicas" in str(ei.value)
