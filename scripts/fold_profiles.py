#!/usr/bin/env python3
"""Fold a finished A/B or measurement directory under profiles/ into one archive file plus its README.

Every round's A/B left dozens of 4-line logs per directory (1,031 tracked files).  This keeps all of the
evidence -- byte for byte -- but as ONE ``raw_logs.txt`` per directory, each original file introduced by a
``==== <relative path> (<n> bytes) ====`` header, so ``profiles/r5/dma_place/run3.log`` becomes section ``run3.log`` of
``profiles/r5/dma_place/raw_logs.txt``.  ``README.md``, ``summary*.txt`` / ``pmc.txt`` and every file some document or
source cites by path stay as they are.  Binary files are left alone.

    python scripts/fold_profiles.py profiles/r5/dma_place profiles/r5/wgrad16 ...
    python scripts/fold_profiles.py --unfold profiles/r5/dma_place      # restore the original files
"""
from __future__ import annotations

import argparse
import os
import sys

KEEP = ("README.md", "pmc.txt")
ARCHIVE = "raw_logs.txt"
SEP = "==== "


def _keep(name: str) -> bool:
    return name in KEEP or (name.startswith("summary") and name.endswith(".txt")) or name == ARCHIVE


def _text(path: str):
    with open(path, "rb") as fh:
        data = fh.read()
    try:
        return data.decode("utf-8")
    except UnicodeDecodeError:
        return None


def cited_paths(roots=("README.md", "BASELINE.md", "SURVEY.md", "docs", "distributed_pytorch_hpc_amd", "benchmarks",
                        "scripts", "tests", "profiles", "bench.py", "__graft_entry__.py")) -> set:
    """Every profiles/... path that a document or source file cites: those files stay where they are."""
    import re

    out = set()
    for root in roots:
        walk = os.walk(root) if os.path.isdir(root) else [("", None, [root])]
        for dp, _, fs in walk:
            for f in fs:
                p = os.path.join(dp, f)
                if p.endswith((".md", ".py", ".hip", ".h", ".cpp", ".sh", ".txt")) and os.path.isfile(p):
                    with open(p, errors="ignore") as fh:
                        out.update(c.rstrip("./") for c in re.findall(r"profiles/[A-Za-z0-9_./-]+", fh.read()))
    return out


def fold(d: str, keep: set = frozenset()) -> int:
    parts = []
    for root, _, files in sorted(os.walk(d)):
        for f in sorted(files):
            p = os.path.join(root, f)
            rel = os.path.relpath(p, d)
            if (root == d and _keep(f)) or os.path.normpath(p) in keep:
                continue
            t = _text(p)
            if t is None:
                continue
            parts.append((rel, p, t))
    if not parts:
        return 0
    arch = os.path.join(d, ARCHIVE)
    mode = "a" if os.path.exists(arch) else "w"
    with open(arch, mode) as fh:
        for rel, _, t in parts:
            fh.write(f"{SEP}{rel} ({len(t.encode())} bytes) ====\n{t}")
            if not t.endswith("\n"):
                fh.write("\n")
    for _, p, _ in parts:
        os.remove(p)
    for root, dirs, files in sorted(os.walk(d, topdown=False)):
        if root != d and not os.listdir(root):
            os.rmdir(root)
    return len(parts)


def unfold(d: str) -> int:
    arch = os.path.join(d, ARCHIVE)
    with open(arch) as fh:
        lines = fh.read().split("\n")
    n, cur, size, buf = 0, None, 0, []

    def flush():
        nonlocal n
        if cur is None:
            return
        p = os.path.join(d, cur)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        body = "\n".join(buf)
        if len((body + "\n").encode()) <= size:   # the original ended with a newline (the header records its size)
            body += "\n"
        with open(p, "w") as out:
            out.write(body)
        n += 1

    for ln in lines:
        if ln.startswith(SEP) and ln.endswith(" bytes) ===="):
            flush()
            name, tail = ln[len(SEP):].rsplit(" (", 1)
            cur, size, buf = name, int(tail.split()[0]), []
        else:
            buf.append(ln)
    flush()
    os.remove(arch)
    return n


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--unfold", action="store_true")
    a = ap.parse_args(argv)
    keep = set() if a.unfold else {os.path.normpath(c) for c in cited_paths()}
    for d in a.dirs:
        n = unfold(d) if a.unfold else fold(d, keep)
        print(f"{d}: {'restored' if a.unfold else 'folded'} {n} file(s)", file=sys.stderr)


if __name__ == "__main__":
    main()
