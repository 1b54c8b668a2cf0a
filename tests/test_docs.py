"""Evidence hygiene: every `profiles/...` path the design
documents cite exists in the tree (brace lists `{3,5}` and trailing ranges like
`r03ab7-9` expanded)."""
import itertools
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md", "profiles/r06/README.md", "tools/README.md"]


def _expand(p):
    m = re.search(r"\{([^}]*)\}", p)
    if m:
        return list(itertools.chain.from_iterable(
            _expand(p[:m.start()] + alt + p[m.end():]) for alt in m.group(1).split(",")))
    r = re.match(r"(.*?)(\d+)-(\d+)$", p)
    if r and int(r.group(3)) > int(r.group(2)):
        return [f"{r.group(1)}{i}" for i in range(int(r.group(2)), int(r.group(3)) + 1)]
    return [p]


def test_cited_profile_paths_exist():
    missing = []
    for doc in DOCS:
        path = os.path.join(ROOT, doc)
        if not os.path.exists(path):
            continue
        text = open(path, encoding="utf-8").read()
        for m in set(re.findall(r"profiles/[A-Za-z0-9_./:{},\-]+", text)):
            p = m.rstrip(".,:;)`")
            for q in _expand(p):
                if not os.path.exists(os.path.join(ROOT, q)):
                    missing.append(f"{doc}: {q}")
    assert not missing, "\n".join(sorted(missing))
