"""Every ``profiles/...`` path the docs cite (README.md,
docs/*.md, profiles/README.md) names at least one tracked file, and the
evidence tree stays small enough to read (verdict r5: 1,978 tracked files,
mostly raw per-run JSON; the per-run files nothing cites were pruned with
``scripts/profile_citations.py --prune``)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import pytest  # noqa: E402

import profile_citations as pc  # noqa: E402

# The GPU-box snapshot leaves the evidence tree out (.gpurunignore): nothing
# to resolve there.
needs_tree = pytest.mark.skipif(not os.path.isdir(os.path.join(ROOT, "profiles")),
                                reason="no profiles/ in this tree (GPU-box snapshot)")


@needs_tree
def test_every_cited_profile_path_resolves():
    bad = pc.check()
    assert not bad, "\n".join(f"{c} (cited in {', '.join(sorted(d))})" for c, d in sorted(bad.items()))


def test_resolver_expands_braces_globs_and_directories():
    files = ["profiles/r05/b02/ttft1_bp0.json", "profiles/r05/b02/ttft8_bp250.json", "profiles/r05/b13/x/summary.txt"]
    assert pc.resolve("profiles/r05/b02/ttft{1,8}_bp{0,250}.json", files) == files[:2]
    assert pc.resolve("profiles/r05/b02/ttft*_bp0.json", files) == files[:1]
    assert pc.resolve("profiles/r05/b13/", files) == files[2:]
    assert pc.resolve("profiles/r05/b14/", files) == []


@needs_tree
def test_profiles_tree_is_pruned():
    assert len(pc.tracked()) <= 500
