"""Every bench line's roofline.traffic comes from a committed rocprofv3 summary
(benchlines/common.py `_pmc_traffic`), which returns None when the summary's
kernel name does not match the one the line names.  A kernel renamed by a new
template argument would silently drop `traffic` from the line; this keeps every
reference resolvable (CPU only: reads the committed profiles)."""
import ast
import json
import os

from conftest import ROOT

SOURCES = ["bench.py"] + [os.path.join("benchlines", f) for f in sorted(os.listdir(os.path.join(ROOT, "benchlines")))
                          if f.endswith(".py")]


def _namespace():
    import benchlines.common as common
    import benchlines.zipf as zipf
    ns = {k: getattr(common, k) for k in dir(common) if k.isupper()}
    ns.update({k: getattr(zipf, k) for k in dir(zipf) if k.isupper()})
    return ns


def _calls():
    out = []
    for rel in SOURCES:
        with open(os.path.join(ROOT, rel)) as fh:
            tree = ast.parse(fh.read(), rel)
        for node in ast.walk(tree):
            if isinstance(node, ast.Call) and getattr(node.func, "id", None) == "_pmc_traffic":
                out.append((rel, node.args[0], node.args[1]))
    return out


def test_every_line_traffic_reference_resolves():
    ns = _namespace()
    calls = _calls()
    assert len(calls) >= 6, calls  # headline, Zipf, device compaction, block verify, packet, EC
    for rel, a_path, a_kernel in calls:
        path = eval(compile(ast.Expression(a_path), rel, "eval"), dict(ns))
        kernel = eval(compile(ast.Expression(a_kernel), rel, "eval"), dict(ns))
        with open(os.path.join(ROOT, path)) as fh:
            pmc = json.load(fh)
        assert pmc.get("kernel") == kernel, (rel, path, pmc.get("kernel"), kernel)
        assert pmc.get("traffic_bytes_per_launch"), (rel, path)
        assert 0.99 < pmc["traffic_bytes_per_launch"] / pmc["algorithmic_bytes_per_launch"] < 1.05, (rel, path)
