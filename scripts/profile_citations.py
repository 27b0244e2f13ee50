#!/usr/bin/env python3
"""Evidence paths cited by the docs, resolved against the tracked tree.

The docs (README.md, docs/*.md, profiles/README.md) cite raw
evidence as ``profiles/...`` paths: files, directories (a trailing ``/`` or a
path that is a directory in the tree), shell globs (``*``) and brace lists
(``{a,b}``). ``resolve()`` expands one citation into the tracked files it
names; ``check()`` lists the citations that name nothing (the test
tests/test_profiles_cited.py keeps that list empty). ``keep_set()`` is what
``--prune`` keeps: every file a citation names exactly, the summaries of every
cited directory (summary.*, *.md, box.json, plan.txt), a few files of a cited
directory that has no summary, and every summary in the tree; the rest of the
per-run JSON is removed from git (it stays in the history).

    python scripts/profile_citations.py            # report unresolved citations
    python scripts/profile_citations.py --prune    # git rm what nothing cites
"""
from __future__ import annotations

import argparse
import fnmatch
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"profiles/[A-Za-z0-9_.\-/{},*]+")
# profiles/README.md names its files relative to profiles/ (`r05/b11/nodeprof/`).
REL = re.compile(r"`(r\d\d/[A-Za-z0-9_.\-/{},*]+)`")
# Placeholders in prose, not paths.
PLACEHOLDERS = ("profiles/r05/bNN", "profiles/r06/bNN")


def doc_files() -> list[str]:
    out = ["BASELINE.md", "README.md", "profiles/README.md"] + sorted(glob.glob(os.path.join(ROOT, "docs", "*.md")))
    return [os.path.relpath(os.path.join(ROOT, f), ROOT) for f in out if os.path.isfile(os.path.join(ROOT, f))]


def tracked() -> list[str]:
    """Tracked files under profiles/ (the files on disk where there is no git checkout)."""
    try:
        r = subprocess.run(["git", "ls-files", "profiles"], cwd=ROOT, capture_output=True, text=True)
        if r.returncode == 0 and r.stdout.strip():
            return r.stdout.split()
    except OSError:
        pass
    out = []
    for d, _, fs in os.walk(os.path.join(ROOT, "profiles")):
        out += [os.path.relpath(os.path.join(d, f), ROOT) for f in fs]
    return sorted(out)


def citations(files: list[str] | None = None) -> dict[str, set[str]]:
    cites: dict[str, set[str]] = {}
    for f in files or doc_files():
        with open(os.path.join(ROOT, f), errors="ignore") as fh:
            text = fh.read()
            found = PAT.findall(text)
            if f == "profiles/README.md":
                found += ["profiles/" + m for m in REL.findall(text)]
            for m in found:
                m = m.rstrip(".,;:)`'\"")
                if m.startswith(PLACEHOLDERS):
                    continue
                cites.setdefault(m, set()).add(f)
    return cites


def expand_braces(p: str) -> list[str]:
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return [p]
    out = []
    for alt in m.group(1).split(","):
        out += expand_braces(p[:m.start()] + alt + p[m.end():])
    return out


def resolve(c: str, files: list[str]) -> list[str]:
    hits: list[str] = []
    for p in expand_braces(c):
        p = p.rstrip("/")
        if "*" in p:
            hits += [f for f in files if fnmatch.fnmatch(f, p) or fnmatch.fnmatch(f, p + "/*")]
        else:
            hits += [f for f in files if f == p or f.startswith(p + "/")]
    return sorted(set(hits))


def is_summary(f: str) -> bool:
    b = os.path.basename(f)
    return b.startswith("summary") or b.endswith(".md") or b in ("box.json", "plan.txt", "README.md")


def check(files: list[str] | None = None) -> dict[str, set[str]]:
    """Citations that resolve to no tracked file, with the docs citing them."""
    t = tracked() if files is None else files
    return {c: d for c, d in citations().items() if not resolve(c, t)}


def keep_set(files: list[str]) -> set[str]:
    keep = {f for f in files if is_summary(f)}
    for c in citations():
        hits = resolve(c, files)
        exact = [h for h in hits if h == c.rstrip("/")]
        if exact or len(hits) <= 6:
            keep.update(hits)
            continue
        sums = [h for h in hits if is_summary(h)]
        keep.update(sums or sorted(hits, key=lambda h: os.path.getsize(os.path.join(ROOT, h)))[:3])
    return keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prune", action="store_true")
    a = ap.parse_args()
    files = tracked()
    bad = check(files)
    for c, d in sorted(bad.items()):
        print(f"unresolved: {c}  (cited in {', '.join(sorted(d))})")
    if a.prune:
        keep = keep_set(files)
        drop = [f for f in files if f not in keep]
        print(f"tracked {len(files)}, keep {len(keep)}, drop {len(drop)}")
        for i in range(0, len(drop), 200):
            subprocess.run(["git", "rm", "-q", "--cached", "--"] + drop[i:i + 200], cwd=ROOT, check=True)
            for f in drop[i:i + 200]:
                os.remove(os.path.join(ROOT, f))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
