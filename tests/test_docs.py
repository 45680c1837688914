"""DESIGN.md describes the current design with evidence that exists: every repository path
it cites (profiles/, scripts/, tests/, oracle/, include/) resolves, and every test it names by
function is defined. CPU only."""
import os
import re

from conftest import PKG, REPO


def _design():
    return open(os.path.join(REPO, "DESIGN.md")).read()


def test_design_cites_existing_files():
    t = _design()
    paths = set(re.findall(r"\b((?:profiles|scripts|tests|oracle|include)/[A-Za-z0-9_./-]+)", t))
    missing = []
    for p in sorted(paths):
        p = p.rstrip(".,")
        if p.endswith("/"):
            p = p[:-1]
        if p.endswith("_"):  # a glob in the text (`tests/golden/metrics_*.npz`)
            import glob
            if glob.glob(os.path.join(REPO, p + "*")):
                continue
        if not any(os.path.exists(os.path.join(root, p)) for root in (REPO, PKG)):
            missing.append(p)
    assert not missing, missing


def test_design_names_existing_tests():
    t = _design()
    names = set()
    for root, _, files in os.walk(os.path.join(REPO, "tests")):
        for f in files:
            if f.endswith(".py"):
                names |= set(re.findall(r"def (test_[a-z0-9_]+)", open(os.path.join(root, f)).read()))
    cited = set(re.findall(r"\b(test_[a-z0-9_]+)\b", t)) - {n for n in re.findall(r"tests/(test_[a-z0-9_]+)\.py", t)}
    assert not (cited - names), sorted(cited - names)
