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


# ---- precedence and associativity: a random expression printed with the fewest parentheses CEL's
# precedence allows must evaluate like the same tree printed fully parenthesised
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3,
         "+": 4, "-": 4, "*": 5, "/": 5, "%": 5}


@st.composite
def _int_expr(draw, depth=0):
    if depth > 3 or draw(st.integers(0, 3)) == 0:
        return ("lit", draw(st.integers(-20, 20)))
    op = draw(st.sampled_from(["+", "-", "*", "/", "%"]))
    return ("bin", op, draw(_int_expr(depth + 1)), draw(_int_expr(depth + 1)))


@st.composite
def _bool_expr(draw, depth=0):
    kind = draw(st.integers(0, 3 if depth < 2 else 1))
    if kind <= 1:
        return ("bin", draw(st.sampled_from(["==", "!=", "<", "<=", ">", ">="])),
                draw(_int_expr(2)), draw(_int_expr(2)))
    if kind == 2:
        return ("not", draw(_bool_expr(depth + 1)))
    return ("bin", draw(st.sampled_from(["&&", "||"])), draw(_bool_expr(depth + 1)),
            draw(_bool_expr(depth + 1)))


def _full(e) -> str:
    if e[0] == "lit":
        return f"({e[1]})" if e[1] < 0 else str(e[1])
    if e[0] == "not":
        return f"(!{_full(e[1])})"
    return f"({_full(e[2])} {e[1]} {_full(e[3])})"


def _minimal(e, parent: int = 0, right: bool = False) -> str:
    if e[0] == "lit":
        return f"({e[1]})" if e[1] < 0 else str(e[1])
    if e[0] == "not":
        return "!" + _minimal(e[1], 9)
    p = _PREC[e[1]]
    s = f"{_minimal(e[2], p)} {e[1]} {_minimal(e[3], p, True)}"
    # left-associative: a right operand of equal precedence keeps its parentheses; so does any
    # comparison operand of a comparison (CEL relations do not chain)
    need = p < parent or (p == parent and right) or (p == parent == 3)
    return f"({s})" if need else s


@settings(max_examples=300, deadline=None)
@given(st.one_of(_int_expr(), _bool_expr()))
def test_precedence_matches_full_parenthesisation(e):
    def run(src):
        try:
            return ("ok", cel.evaluate(src, {}))
        except cel.CelError as err:
            return ("err", type(err).__name__)
    assert run(_minimal(e)) == run(_full(e)), (_minimal(e), _full(e))
