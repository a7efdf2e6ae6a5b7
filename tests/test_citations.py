"""Reference citations (``File.ext:line`` / ``File.ext:a-b``) in the boundary
header, INTEGRATION.md and the sources point at lines that exist, and the
boundary's method / type citations point at the declarations they name.
Line counts and declaration lines come from tests/golden/reference_lines.json
(numbers only); when /root/reference is present the fixture itself is
re-derived and compared."""
import glob
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "reference_lines.json")
REF = "/root/reference/PathTracerAP"

with open(FIXTURE) as _f:
    REFLINES = json.load(_f)["files"]

CITE = re.compile(r"\b([A-Za-z_]+\.(?:h|cpp)):(\d+)(?:-(\d+))?")
SOURCES = (["include/pathtracer_amd.h", "INTEGRATION.md", "DESIGN.md", "bench.py", "__graft_entry__.py"]
           + sorted(glob.glob(os.path.join(ROOT, "pathtracerap_amd", "csrc", "*.*")))
           + sorted(glob.glob(os.path.join(ROOT, "pathtracerap_amd", "*.py")))
           + sorted(glob.glob(os.path.join(ROOT, "oracle", "*.[ch]")))
           + sorted(glob.glob(os.path.join(ROOT, "oracle", "*.py")))
           + sorted(glob.glob(os.path.join(ROOT, "tests", "*.py"))))


def citations(path):
    full = path if os.path.isabs(path) else os.path.join(ROOT, path)
    with open(full, encoding="utf-8") as f:
        for n, line in enumerate(f, 1):
            for m in CITE.finditer(line):
                if m.group(1) in REFLINES:
                    a = int(m.group(2))
                    yield n, line, m.group(1), a, int(m.group(3)) if m.group(3) else a


@pytest.mark.parametrize("path", SOURCES, ids=lambda p: os.path.relpath(p, ROOT) if os.path.isabs(p) else p)
def test_citations_within_reference_files(path):
    bad = [f"{os.path.basename(path)}:{n}: {f}:{a}-{b} (file has {REFLINES[f]['lines']} lines)"
           for n, _, f, a, b in citations(path) if not (1 <= a <= b <= REFLINES[f]["lines"])]
    assert not bad, "\n".join(bad)


# declarations whose citations are checked by name: the Renderer methods the C ABI
# replaces and the enums it restates (other names also appear as field types)
CHECKED = {"Renderer.h": ["allocateOnGPU", "renderLoop", "renderImage", "free"],
           "Primitive.h": ["MaterialType", "EntityType"], "Scene.h": ["Scene(string config)"]}


def _qualified(f, name):
    """How a declaration is named in our text: Renderer.h methods as Renderer::m."""
    if f == "Renderer.h":
        return "Renderer::" + name
    return name


@pytest.mark.parametrize("path", ["include/pathtracer_amd.h", "INTEGRATION.md",
                                  "pathtracerap_amd/csrc/scene.h", "pathtracerap_amd/csrc/pt_types.h"])
def test_boundary_citations_name_their_declarations(path):
    """A line that names a mapped declaration and cites its file must cite a
    range holding that declaration's line."""
    bad = []
    for n, line, f, a, b in citations(path):
        for name in CHECKED.get(f, []):
            at = REFLINES[f]["symbols"][name]
            key = _qualified(f, name)
            if re.search(r"(?<![\w:])" + re.escape(key) + r"(?![\w(])", line) and not (a <= at <= b):
                # the line may cite the same file once per declaration it names
                others = [(a2, b2) for _, _, f2, a2, b2 in citations_in_line(line) if f2 == f]
                if not any(a2 <= at <= b2 for a2, b2 in others):
                    bad.append(f"{path}:{n}: {key} is at {f}:{at}, cited {f}:{a}-{b}")
    assert not bad, "\n".join(sorted(set(bad)))


def citations_in_line(line):
    for m in CITE.finditer(line):
        if m.group(1) in REFLINES:
            a = int(m.group(2))
            yield 0, line, m.group(1), a, int(m.group(3)) if m.group(3) else a


def test_boundary_header_cites_every_renderer_method():
    with open(os.path.join(ROOT, "include", "pathtracer_amd.h")) as f:
        text = f.read()
    for name, at in REFLINES["Renderer.h"]["symbols"].items():
        if not name.startswith("class "):
            assert f"Renderer.h:{at}" in text, f"Renderer::{name} (Renderer.h:{at}) not cited"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_fixture_matches_reference():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mkref", os.path.join(ROOT, "tests", "golden", "make_reference_lines.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    assert mk.scan(REF)["files"] == REFLINES
