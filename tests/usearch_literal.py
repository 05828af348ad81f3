"""Literal transcription of usearch's HNSW loops (TEST INFRASTRUCTURE ONLY).

The reference reaches unum-cloud/usearch through `usearch::Index::{add,
remove, search}` (/root/reference/src/index/usearch.rs:215, 221, 245, 276);
the library is not vendored.  This module restates, loop for
loop, the published v2-series index.hpp routines the C oracle restates in set
form -- two binary heaps (`next`: min-heap of candidates to expand, `top`:
max-heap of the best `top_limit`), distance-only comparisons, usearch's own
break / admission conditions:

  search_for_one_            greedy descent, strict `<` improvement in row order
  search_to_insert_          break: nearest of next > radius AND top full
  search_to_find_in_base_    break: nearest of next > radius; the `allow`
                             predicate (index_dense: key != free_key_) keeps a
                             removed successor out of `top` after it was pushed
                             to `next`; the start joins `top` only if allowed
  refine_                    sort ascending; fewer than `needed` => all; else
                             keep c unless dist(c, kept) < c.distance
  connect_new_node_          refine_(connectivity) on every level
  reconnect_neighbor_nodes_  append below connectivity_max (level ? M : M0),
                             else refine_(connectivity_max) over the row + new;
                             a row already holding the new node is left as is
  index_dense add_ / update  removed slots queue in free_keys_ (a FIFO ring);
                             an add pops the oldest and re-links it in place
                             (index_gt::update: rows cleared, level kept,
                             other nodes' links into it kept), else appends.
                             The node is never its own candidate; the entry
                             point's slot is not reused while it is the entry
                             (see oracle/vsg_oracle.h orc_hnsw_add)

Distances come from the oracle's f32 metric (oracle.distance), so on float data
without exact ties the set formulation (oracle/vsg_oracle.c beam(),
beam_filtered(), select_heuristic()) must produce the same graph and results;
tests/test_oracle.py::test_oracle_matches_literal_usearch_loops checks it.
Pure Python: small graphs only.
"""
from __future__ import annotations

import heapq
from collections import deque

import numpy as np

import oracle as O


class LiteralHnsw:
    def __init__(self, dim, metric, connectivity, expansion_add, seed=0):
        self.dim, self.metric = dim, metric
        self.M, self.M0, self.efc, self.seed = connectivity, 2 * connectivity, expansion_add, seed
        self.vecs: list[np.ndarray] = []
        self.levels: list[int] = []
        self.links: list[list[list[int]]] = []  # links[slot][level] = ordered neighbours
        self.removed: set[int] = set()
        self.free: deque[int] = deque()  # index_dense free_keys_, oldest removal first
        self.entry, self.max_level = 0xFFFFFFFF, -1

    def _d(self, a, b) -> float:
        return O.distance(self.metric, a, b)

    # search_for_one_: greedy on levels begin_level .. end_level + 1
    def _search_for_one(self, q, closest, begin, end, exclude=None):
        cd = self._d(q, self.vecs[closest])
        for level in range(begin, end, -1):
            changed = True
            while changed:
                changed = False
                for c in self.links[closest][level]:
                    if c == exclude:     # never its own candidate
                        continue
                    d = self._d(q, self.vecs[c])
                    if d < cd:
                        cd, closest, changed = d, c, True
        return closest

    # search_to_insert_ -> top as a list of (distance, slot)
    def _search_to_insert(self, q, start, new, level, top_limit):
        r = self._d(q, self.vecs[start])
        nxt = [(r, start)]               # min-heap
        top = [(-r, start)]              # max-heap via negation
        visited = {start, new}           # `new` is never its own candidate
        while nxt:
            cd, cs = nxt[0]
            if cd > -top[0][0] and len(top) == top_limit:
                break
            heapq.heappop(nxt)
            if cs == new:
                continue
            for s in self.links[cs][level]:
                if s in visited:
                    continue
                visited.add(s)
                d = self._d(q, self.vecs[s])
                if len(top) < top_limit or d < -top[0][0]:
                    heapq.heappush(nxt, (d, s))
                    heapq.heappush(top, (-d, s))
                    if len(top) > top_limit:
                        heapq.heappop(top)
        return [(-nd, s) for nd, s in top]

    def _refine(self, cands, needed):
        top = sorted(cands)
        if len(top) < needed:
            return [s for _, s in top]
        kept = [top[0]]
        for cd, cs in top[1:]:
            if all(not (self._d(self.vecs[cs], self.vecs[ks]) < cd) for _, ks in kept):
                kept.append((cd, cs))
                if len(kept) == needed:
                    break
        return [s for _, s in kept]

    def add(self, slot, vec):
        assert slot == len(self.vecs)
        self._append(vec)
        self._connect(slot)

    def _append(self, vec):
        slot = len(self.vecs)
        L = O.sample_level(self.seed, slot, self.M)
        self.vecs.append(np.ascontiguousarray(vec, np.float32))
        self.levels.append(L)
        self.links.append([[] for _ in range(L + 1)])
        return slot

    def add_one(self, vec):
        """index_dense add_ of one vector: pop the oldest free slot (the entry
        point's is skipped and keeps its place) and run index_gt::update on it --
        new vector, rows cleared, level kept, live again, re-linked -- or append
        when none is free.  Returns the slot."""
        s = None
        for i, f in enumerate(self.free):
            if f != self.entry:
                s = f
                del self.free[i]
                break
        if s is None:
            s = self._append(vec)
        else:
            self.vecs[s] = np.ascontiguousarray(vec, np.float32)
            self.links[s] = [[] for _ in range(self.levels[s] + 1)]
            self.removed.discard(s)
        self._connect(s)
        return s

    def add_batch(self, vecs):
        """One multi-key add call = that many single adds in call order (each
        pops one free slot and re-links it before the next key's slot is
        touched).  Returns the slots in call order."""
        return [self.add_one(v) for v in vecs]

    def replace(self, slot_of, key, vec):
        """The reference's AddOrReplace of one message (usearch.rs:214-221):
        remove the key's live slot if any, then add.  slot_of: key -> slot map
        (updated); returns the new slot."""
        if key in slot_of:
            self.remove([slot_of.pop(key)])
        s = self.add_one(vec)
        slot_of[key] = s
        return s

    # connect_node_across_levels_ (index_gt::add / update)
    def _connect(self, slot):
        vec, L = self.vecs[slot], self.levels[slot]
        if self.entry == 0xFFFFFFFF:
            self.entry, self.max_level = slot, L
            return
        closest = self._search_for_one(vec, self.entry, self.max_level, L, exclude=slot)
        for level in range(min(L, self.max_level), -1, -1):
            top = self._search_to_insert(vec, closest, slot, level, self.efc)
            self.links[slot][level] = self._refine(top, self.M)          # connect_new_node_
            closest = self.links[slot][level][0]
            cmax = self.M if level else self.M0                          # reconnect_neighbor_nodes_
            for c in self.links[slot][level]:
                row = self.links[c][level]
                if slot in row:                  # already present: nothing changes
                    continue
                if len(row) < cmax:
                    row.append(slot)
                    continue
                cands = [(self._d(vec, self.vecs[c]), slot)]
                cands += [(self._d(self.vecs[c], self.vecs[s]), s) for s in row]
                self.links[c][level] = self._refine(cands, cmax)
        if L > self.max_level:
            self.entry, self.max_level = slot, L

    def remove(self, slots):
        for s in slots:
            s = int(s)
            if s not in self.removed:
                self.removed.add(s)
                self.free.append(s)      # index_dense_gt::remove: free_keys_.push(slot)

    # index_dense search: search_for_one_ to level 0, then search_to_find_in_base_
    def search(self, q, k, ef):
        if self.entry == 0xFFFFFFFF:
            return [], []
        q = np.ascontiguousarray(q, np.float32)
        top_limit = max(ef, k)
        start = self._search_for_one(q, self.entry, self.max_level, 0)
        radius = self._d(q, self.vecs[start])
        nxt = [(radius, start)]
        top = [] if start in self.removed else [(-radius, start)]
        visited = {start}
        while nxt:
            cd, cs = nxt[0]
            if cd > radius:
                break
            heapq.heappop(nxt)
            for s in self.links[cs][0]:
                if s in visited:
                    continue
                visited.add(s)
                d = self._d(q, self.vecs[s])
                if len(top) < top_limit or d < radius:
                    heapq.heappush(nxt, (d, s))
                    if s in self.removed:   # the `allow` predicate
                        continue
                    heapq.heappush(top, (-d, s))
                    if len(top) > top_limit:
                        heapq.heappop(top)
                    radius = -top[0][0]
        res = sorted((-nd, s) for nd, s in top)[:k]
        return [s for _, s in res], [d for d, _ in res]
