#pragma once
// Strand schedule shared by the R1CS and sparse-R1CS solvers (solver.hip,
// scs_solver.hip).  gnark solves level by level (constraint/<curve>/solver.go:
// 418-533: r1cs.Levels, a level's constraints in parallel over the CPU cores);
// on the GPU a level of a chain circuit is one wave per SIMD walking one
// dependent constraint, so the launches are latency-bound.  The schedule:
//   * in Levels order, each constraint's unknown term (the single term whose
//     wire neither the inputs nor an earlier constraint produced) and the
//     producer of every wire;
//   * greedy chains: a constraint extends the strand whose tail produced one of
//     its inputs (the most recent such tail);
//   * super-levels: sl(c) = max(sl(previous in its strand), sl(d) + 1 for
//     every dependency d on another strand).
// One launch per super-level, a thread per strand segment, walking its
// constraints in order; values produced by other strands were written by
// earlier launches.  Returns false when the levels do not match the system
// (two unknown terms, or an input produced at the same or a later level): the
// caller then runs the level launches, whose kernel reports the error.
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

namespace gg {

struct StrandPlan {
    std::vector<uint32_t> unk;         // per constraint: term id of its unknown, ~0 = none
    std::vector<uint32_t> order;       // constraints by (super-level, strand, level position)
    std::vector<uint32_t> seg_start;   // segment s = order[seg_start[s], seg_start[s+1])
    std::vector<uint32_t> sl_seg_off;  // segments of super-level l: [sl_seg_off[l], sl_seg_off[l+1])
};

// terms(c, f) calls f(term_id, wire) for every term of constraint c; wires
// below nin (ONE_WIRE / the witness) are solved up front.  skip(c): the
// constraint solves nothing and is left out (SCS commitment rows).
template <class Terms, class Skip>
bool build_strand_plan(size_t nc, size_t nw, uint32_t nin, const std::vector<uint32_t>& level_off,
                       const std::vector<uint32_t>& level_cons, Terms terms, Skip skip, StrandPlan& plan) {
    const uint32_t NONE = 0xffffffffu;
    std::vector<uint32_t> lev(nc, NONE), prod(nw, NONE);
    plan.unk.assign(nc, NONE);
    for (size_t l = 0; l + 1 < level_off.size(); l++)
        for (uint32_t i = level_off[l]; i < level_off[l + 1]; i++) lev[level_cons[i]] = (uint32_t)l;
    std::vector<uint32_t> strand(nc), sl(nc), tail, deps;
    std::vector<std::pair<uint64_t, uint32_t>> key;  // ((sl, strand), position) -> order
    std::vector<uint32_t> cons;
    key.reserve(nc);
    cons.reserve(nc);
    bool ok = true;
    for (size_t l = 0; ok && l + 1 < level_off.size(); l++) {
        for (uint32_t i = level_off[l]; ok && i < level_off[l + 1]; i++) {
            const uint32_t c = level_cons[i];
            if (skip(c)) continue;
            deps.clear();
            uint32_t u = NONE, uw = NONE;
            terms(c, [&](uint32_t t, uint32_t w) {
                if (w < nin || !ok) return;
                const uint32_t p = prod[w];
                if (p == NONE) {
                    if (u != NONE) ok = false;  // two unknown terms
                    u = t;
                    uw = w;
                } else if (p != c) {
                    if (lev[p] >= l) ok = false;  // produced in this or a later level
                    deps.push_back(p);
                }
            });
            if (!ok) break;
            if (u != NONE) prod[uw] = c;
            plan.unk[c] = u;
            uint32_t best = NONE;
            for (uint32_t d : deps)
                if (tail[strand[d]] == d && (best == NONE || lev[d] > lev[best])) best = d;
            uint32_t s, level = 0;
            if (best != NONE) {
                s = strand[best];
                level = sl[best];
            } else {
                s = (uint32_t)tail.size();
                tail.push_back(NONE);
            }
            for (uint32_t d : deps)
                if (strand[d] != s) level = std::max(level, sl[d] + 1);
            strand[c] = s;
            tail[s] = c;
            sl[c] = level;
            key.push_back({((uint64_t)level << 32) | s, i});
            cons.push_back(c);
        }
    }
    if (!ok) return false;
    std::vector<uint32_t> idx(cons.size());
    for (size_t k = 0; k < idx.size(); k++) idx[k] = (uint32_t)k;
    std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    plan.order.resize(idx.size());
    plan.seg_start.clear();
    plan.sl_seg_off.clear();
    uint64_t prev = ~0ull;
    uint32_t cur_sl = NONE;
    for (size_t k = 0; k < idx.size(); k++) {
        plan.order[k] = cons[idx[k]];
        const uint64_t kk = key[idx[k]].first;
        if (kk != prev) {
            const uint32_t lvl = (uint32_t)(kk >> 32);
            while (cur_sl == NONE || cur_sl < lvl) {
                plan.sl_seg_off.push_back((uint32_t)plan.seg_start.size());
                cur_sl = cur_sl == NONE ? 0 : cur_sl + 1;
            }
            plan.seg_start.push_back((uint32_t)k);
            prev = kk;
        }
    }
    plan.seg_start.push_back((uint32_t)idx.size());
    plan.sl_seg_off.push_back((uint32_t)plan.seg_start.size() - 1);
    return true;
}

}  // namespace gg
