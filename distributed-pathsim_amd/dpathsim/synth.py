"""Synthetic DBLP-shaped graphs.

dblp_large.gexf is absent from the reference snapshot (.MISSING_LARGE_BLOBS:1),
so the large configs use this generator.  It emits the same schema as
dblp/dblp_small.gexf: author / paper / venue (or topic) nodes, ``author_of``
edges author -> paper and ``submit_at`` (or ``has_topic``) paper -> mid.

Recipe (numpy ``default_rng(seed)``, seed 20180417 by default), in this order:
  1. ``mperm = rng.permutation(n_mids)``; mid weights ∝ rank^-mid_alpha.
     APVPA: one venue per paper, ``mperm[rng.choice(n_mids, n_papers, p)]``.
     APTPA: ``1 + min(Poisson(mids_lambda), mids_cap-1)`` topics per paper,
     drawn the same way, deduplicated per paper.
  2. authors per paper ``k = 1 + min(rng.poisson(authors_lambda), authors_cap-1)``.
  3. ``aperm = rng.permutation(n_authors)``; slot authors
     ``aperm[rng.choice(n_authors, sum(k), p ∝ rank^-author_alpha)]``; the
     first n_authors slots are overwritten by ``rng.permutation(n_authors)``
     (every author writes >= 1 paper, so every g > 0); ``rng.shuffle(slots)``.
  4. slot j belongs to paper ``repeat(arange(n_papers), k)[j]``; duplicate
     (author, paper) pairs are kept in the edge list (the engine's distinct
     removes them, as the reference's does).
Node order: authors, papers, mids.  Edge order: all mid edges by paper, then
all author_of edges by paper.
"""
from __future__ import annotations

import numpy as np

from .graph import APTPA, APVPA, Graph, MetaPath

CONFIGS = {
    # name: (n_authors, n_papers, n_mids, metapath, k)
    "config3": (1_000_000, 3_000_000, 5_000, "APVPA", 10),
    "config3_100k": (100_000, 300_000, 5_000, "APVPA", 10),
    "config4": (1_000_000, 3_000_000, 200_000, "APTPA", 10),
    "config5": (3_000_000, 10_000_000, 20_000, "APVPA", 100),
}


def _zipf_p(n, alpha):
    w = np.arange(1, n + 1, dtype=np.float64) ** (-alpha)
    return w / w.sum()


def synth_dblp(n_authors, n_papers, n_mids, seed=20180417, metapath: MetaPath = APVPA,
               mid_alpha=0.8, author_alpha=0.5, authors_lambda=1.5, authors_cap=30,
               mids_lambda=3.0, mids_cap=20):
    if n_papers * 1 < 1 or n_authors < 1 or n_mids < 1:
        raise ValueError("sizes must be positive")
    rng = np.random.default_rng(seed)
    mperm = rng.permutation(n_mids)
    pm = _zipf_p(n_mids, mid_alpha)
    if metapath.mid_type == "venue":
        mid_paper = np.arange(n_papers, dtype=np.int64)
        mid_id = mperm[rng.choice(n_mids, size=n_papers, p=pm)]
    else:
        km = 1 + np.minimum(rng.poisson(mids_lambda, n_papers), mids_cap - 1)
        mid_paper = np.repeat(np.arange(n_papers, dtype=np.int64), km)
        mid_id = mperm[rng.choice(n_mids, size=int(km.sum()), p=pm)]
        key = np.unique(mid_paper * n_mids + mid_id)
        mid_paper, mid_id = key // n_mids, key % n_mids
    k = 1 + np.minimum(rng.poisson(authors_lambda, n_papers), authors_cap - 1)
    total = int(k.sum())
    if total < n_authors:
        raise ValueError("not enough author slots to give every author a paper")
    aperm = rng.permutation(n_authors)
    slots = aperm[rng.choice(n_authors, size=total, p=_zipf_p(n_authors, author_alpha))]
    slots[:n_authors] = rng.permutation(n_authors)
    rng.shuffle(slots)
    paper_of_slot = np.repeat(np.arange(n_papers, dtype=np.int64), k)

    na, npp = n_authors, n_papers
    node_type_idx = np.concatenate([np.zeros(na, np.int32), np.ones(npp, np.int32),
                                    np.full(n_mids, 2, np.int32)])
    type_names = [metapath.author_type, metapath.paper_type, metapath.mid_type]
    src = np.concatenate([na + mid_paper, slots]).astype(np.int32)
    dst = np.concatenate([na + npp + mid_id, na + paper_of_slot]).astype(np.int32)
    rel = np.concatenate([np.ones(len(mid_paper), np.int32), np.zeros(total, np.int32)])
    rel_names = [metapath.rel_ap, metapath.rel_px]
    mid_prefix = metapath.mid_type

    def node_id(i):
        if i < na:
            return f"author_{i}"
        if i < na + npp:
            return f"paper_{i - na}"
        return f"{mid_prefix}_{i - na - npp}"

    def label(i):
        if i < na:
            return f"Author {i}"
        if i < na + npp:
            return f"Paper {i - na}."
        return f"{mid_prefix}_{i - na - npp}"

    return Graph(node_type_idx, type_names, src, dst, rel, rel_names, node_ids=node_id,
                 labels=label)


def synth_config(name, seed=20180417, scale=1.0):
    """Graph for a named SURVEY §8d config (``scale`` shrinks authors/papers)."""
    na, npp, nm, mp, _k = CONFIGS[name]
    na, npp = max(1, int(na * scale)), max(1, int(npp * scale))
    return synth_dblp(na, npp, nm, seed=seed, metapath=APTPA if mp == "APTPA" else APVPA)
