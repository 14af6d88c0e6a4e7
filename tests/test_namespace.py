"""The Polars expression namespace (reference python/polars_matmul/__init__.py:
39-196) against a minimal stand-in ``polars`` module (Polars itself is not
installable in this image).  Checks what the namespace hands to
``map_batches``: the function, ``is_elementwise``, ``return_dtype``, the
flatten branch, and the TypeError on an Expr corpus.  Runs in a subprocess so
the stand-in never leaks into other tests.  CPU only: the captured functions
are called with ``_topk`` / ``_matmul`` replaced by recorders."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import json, sys, types
sys.path.insert(0, %(pkg)r)

pl = types.ModuleType("polars")
class _DT:
    def __init__(self, name, *args):
        self.name, self.args = name, args
    def __eq__(self, o):
        return isinstance(o, _DT) and (self.name, self.args) == (o.name, o.args)
    def __repr__(self):
        return f"{self.name}{self.args if self.args else ''}"
pl.UInt32, pl.Float32, pl.Float64 = _DT("UInt32"), _DT("Float32"), _DT("Float64")
pl.List = lambda inner: _DT("List", inner)
pl.Struct = lambda fields: _DT("Struct", tuple(fields.items()))
pl.Array = lambda inner, n: _DT("Array", inner, n)
class Expr:
    def __init__(self):
        self.calls = []
    def map_batches(self, fn, **kw):
        self.calls.append((fn, kw))
        return ("mapped", kw)
class Series:
    def __init__(self, values, inner):
        self.values, self.dtype = values, types.SimpleNamespace(inner=inner)
    def __len__(self):
        return len(self.values)
    def explode(self):
        return ("exploded", self)
registry = {}
def register_expr_namespace(name):
    def deco(cls):
        registry[name] = cls
        return cls
    return deco
pl.Expr, pl.Series = Expr, Series
pl.api = types.SimpleNamespace(register_expr_namespace=register_expr_namespace)
sys.modules["polars"] = pl

import polars_matmul
out = {"registered": sorted(registry), "version": polars_matmul.__version__}
ns_cls = registry["pmm"]
calls = []
polars_matmul._topk = lambda s, c, k, m: calls.append(("topk", s, len(c), k, m)) or "topk-result"
polars_matmul._matmul = lambda s, c: calls.append(("matmul", s, len(c))) or Series([1], pl.Float32)

corpus32 = Series([[1.0, 0.0]] * 3, pl.Float32)
corpus64 = Series([[1.0, 0.0]] * 5, pl.Float64)
e = Expr(); ns_cls(e).topk(corpus32, k=2)
fn, kw = e.calls[0]
out["topk_kw"] = {"is_elementwise": kw["is_elementwise"], "return_dtype": repr(kw["return_dtype"])}
out["topk_dtype_ok"] = kw["return_dtype"] == pl.List(pl.Struct({"index": pl.UInt32, "score": pl.Float64}))
out["topk_call"] = repr(fn("batch")) and repr(calls[-1])
e = Expr(); ns_cls(e).topk(corpus32, k=7, metric="euclidean"); e.calls[0][0]("b2")
out["topk_call2"] = repr(calls[-1])
try:
    ns_cls(Expr()).topk(Expr(), k=1)
    out["expr_error"] = None
except TypeError as err:
    out["expr_error"] = str(err)
e = Expr(); ns_cls(e).matmul(corpus32)
fn, kw = e.calls[0]
out["mm32"] = {"is_elementwise": kw["is_elementwise"], "ok": kw["return_dtype"] == pl.Array(pl.Float32, 3)}
e = Expr(); ns_cls(e).matmul(corpus64)
out["mm64_ok"] = e.calls[0][1]["return_dtype"] == pl.Array(pl.Float64, 5)
e = Expr(); ns_cls(e).matmul(corpus32, flatten=True)
fn, kw = e.calls[0]
out["flat"] = {"is_elementwise": kw["is_elementwise"], "ok": kw["return_dtype"] == pl.Float32}
r = fn("batch3")
out["flat_result_exploded"] = isinstance(r, tuple) and r[0] == "exploded"
out["flat_call"] = repr(calls[-1])
try:
    ns_cls(Expr()).matmul(Expr())
    out["mm_expr_error"] = None
except TypeError as err:
    out["mm_expr_error"] = str(err)
print(json.dumps(out))
'''


def test_namespace_map_batches_contract():
    code = SCRIPT % {"pkg": os.path.join(ROOT, "polars-matmul_amd")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["registered"] == ["pmm"] and out["version"] == "0.1.4"
    # __init__.py:115-119: elementwise, List[Struct{index: u32, score: f64}]
    assert out["topk_kw"]["is_elementwise"] is True and out["topk_dtype_ok"]
    assert out["topk_call"] == "('topk', 'batch', 3, 2, 'cosine')"
    assert out["topk_call2"] == "('topk', 'b2', 3, 7, 'euclidean')"
    # __init__.py:109-113 / :159-164 error text
    assert out["expr_error"].startswith("corpus must be a Polars Series, not an Expression.")
    assert out["mm_expr_error"].startswith("corpus must be a Polars Series, not an Expression.")
    # __init__.py:166-171, :190: Array[f32|f64, len(corpus)] decided by the corpus
    assert out["mm32"] == {"is_elementwise": True, "ok": True} and out["mm64_ok"]
    # __init__.py:173-187: flatten -> not elementwise, inner dtype, explode()
    assert out["flat"] == {"is_elementwise": False, "ok": True}
    assert out["flat_result_exploded"] and out["flat_call"] == "('matmul', 'batch3', 3)"
