/* Design probe (CPU, not product code): the election's tail computed as per-agent RECORD LISTS by
 * tile-local label correcting instead of one synchronous round per launch.
 *
 * After round T0 every agent v holds L_v = max id within T0 hops.  For t > T0 its value is
 * max{ L_w : d(v, w) <= t - T0 }, a step function of t given by the pareto set of pairs (d, val):
 * v reaches value val at round T0 + d.  The pareto sets are the least fixpoint of
 *   list_v = pareto( {(0, L_v)} u { (d + 1, val) : (d, val) in list_u, u in N(v) } )
 * and any order of relaxations reaches it (every pair is a true "val within d hops" statement), so
 * tiles of cells can run to a local fixpoint on chip and exchange borders between launches.  This
 * probe counts what that costs: launches (global iterations), tile activations, local levels, list
 * lengths -- and checks the derived per-round changes and final leaders against the Jacobi rounds.
 *
 * build: gcc -O2 -fopenmp -shared -fPIC -o tools/librecord_sim.so tools/record_tail_sim.c
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define RMAX 32

typedef struct { int32_t d; int32_t v; } ent_t;

/* pareto insert of (d, val) into list (sorted by d asc, val asc strictly); base (0, b) implicit.
 * returns 1 if the list changed, -1 on overflow */
static int ins(ent_t *l, int *len, int32_t b, int32_t d, int32_t val) {
    /* dominated by base or by an entry with d' <= d and val' >= val? */
    if (val <= b) return 0;
    int n = *len, i;
    for (i = 0; i < n && l[i].d <= d; ++i)
        if (l[i].v >= val) return 0;
    /* i = first entry with d' > d; entries with d' >= d and val' <= val are dominated */
    int j = i;
    /* entries before i with d' == d and val' < val: dominated too */
    int k = i;
    while (k > 0 && l[k - 1].d == d) --k; /* l[k..i) have d' == d and val' < val */
    while (j < n && l[j].v <= val) ++j;   /* l[i..j) have d' > d and val' <= val */
    /* new list: l[0..k) + (d,val) + l[j..n) */
    int newn = k + 1 + (n - j);
    if (newn > RMAX) return -1;
    memmove(&l[k + 1], &l[j], sizeof(ent_t) * (size_t)(n - j));
    l[k].d = d;
    l[k].v = val;
    *len = newn;
    return 1;
}

/* stats out: [0] launches, [1] activations, [2] sum of levels over activations, [3] sum over
 * launches of the max levels in that launch (critical path in levels), [4] max list length,
 * [5] overflow, [6] relaxations (vertex recomputes), [7] edge reads */
long rec_sim(long n, const int64_t *rp, const int32_t *col, const int32_t *L, const uint8_t *mark0,
             const int32_t *tile_of, long ntiles, const int64_t *toff, const int32_t *tmem, int64_t *hist,
             long hist_cap, int32_t *final_leader, int64_t *stats, long max_launches, long delta) {
    ent_t *G = (ent_t *)calloc((size_t)n * RMAX, sizeof(ent_t));
    int32_t *Gn = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    ent_t *G2 = (ent_t *)calloc((size_t)n * RMAX, sizeof(ent_t));
    int32_t *G2n = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    uint8_t *mk = (uint8_t *)malloc((size_t)n);
    uint8_t *mk2 = (uint8_t *)calloc((size_t)n, 1);
    uint8_t *tact = (uint8_t *)calloc((size_t)ntiles, 1);
    uint8_t *tact2 = (uint8_t *)calloc((size_t)ntiles, 1);
    memcpy(mk, mark0, (size_t)n);
    for (long v = 0; v < n; ++v)
        if (mk[v]) tact[tile_of[v]] = 1;
    long launches = 0, acts = 0, lev_sum = 0, crit = 0, maxlen = 0, ovf = 0, relax = 0, edges = 0;
    long crit_wg = 0, crit_tiles = 0;
    int32_t *tlev = (int32_t *)calloc((size_t)ntiles, sizeof(int32_t));
    enum { kG = 256 };
    for (;;) {
        long nact = 0;
        for (long t = 0; t < ntiles; ++t) nact += tact[t];
        if (!nact || launches >= max_launches) break;
        ++launches;
        long launch_max = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : acts, lev_sum, relax, edges, ovf) reduction(max : launch_max, maxlen)
        for (long t = 0; t < ntiles; ++t) {
            if (!tact[t]) continue;
            ++acts;
            const int64_t a0 = toff[t], a1 = toff[t + 1];
            const long m = (long)(a1 - a0);
            /* local working copies live in G2 (own agents only) */
            for (int64_t k = a0; k < a1; ++k) {
                const int32_t v = tmem[k];
                G2n[v] = Gn[v];
                memcpy(&G2[(size_t)v * RMAX], &G[(size_t)v * RMAX], sizeof(ent_t) * (size_t)Gn[v]);
            }
            uint8_t *cur = (uint8_t *)calloc((size_t)m, 1), *nxt = (uint8_t *)calloc((size_t)m, 1);
            long nc = 0;
            for (int64_t k = a0; k < a1; ++k)
                if (mk[tmem[k]]) { cur[k - a0] = 1; ++nc; mk[tmem[k]] = 0; }
            long levels = 0;
            /* local index of an in-tile agent: position in tmem; we need v -> k: use a small search
             * via tile_of + a global loc array would be faster; here a per-tile hash is avoided by
             * scanning rows (agents per tile are few thousand) */
            /* two-phase levels (the GPU kernel's form): every listed agent computes its new list from
             * the lists as they were at the start of the level, then all write */
            ent_t *tmp_l = (ent_t *)malloc(sizeof(ent_t) * RMAX * (size_t)m);
            int32_t *tmp_n = (int32_t *)malloc(sizeof(int32_t) * (size_t)m);
            uint8_t *chg = (uint8_t *)calloc((size_t)m, 1);
            int32_t *stamp = (int32_t *)calloc((size_t)m, sizeof(int32_t)); /* level a slot last changed */
            uint8_t *first = (uint8_t *)calloc((size_t)m, 1);
            uint8_t *deferred = (uint8_t *)calloc((size_t)m, 1);
            const long wb = delta > 0 ? (launches) * delta : 0; /* window bound of this launch */
            for (long k = 0; k < m; ++k) first[k] = cur[k];
            while (nc) {
                ++levels;
                long nn = 0;
                for (long k = 0; k < m; ++k) {
                    chg[k] = 0;
                    if (!cur[k]) continue;
                    const int32_t v = tmem[a0 + k];
                    ++relax;
                    ent_t *lv = &tmp_l[(size_t)k * RMAX];
                    tmp_n[k] = G2n[v];
                    memcpy(lv, &G2[(size_t)v * RMAX], sizeof(ent_t) * (size_t)G2n[v]);
                    int changed = 0;
                    for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                        const int32_t u = col[e];
                        const int in = tile_of[u] == t;
                        if (!first[k]) { /* filtered pull: only in-tile neighbours changed last level */
                            if (!in) continue;
                            long lo = 0, hi = m;
                            while (lo < hi) { long md = (lo + hi) / 2; if (tmem[a0 + md] < u) lo = md + 1; else hi = md; }
                            if (stamp[lo] != levels - 1) continue;
                        }
                        ++edges;
                        const ent_t *lu = in ? &G2[(size_t)u * RMAX] : &G[(size_t)u * RMAX];
                        const int32_t nu = in ? G2n[u] : Gn[u];
                        int r = (wb && 1 > wb) ? 0 : ins(lv, &tmp_n[k], L[v], 1, L[u]);
                        if (r < 0) { ++ovf; r = 0; }
                        changed |= r;
                        for (int32_t i = 0; i < nu; ++i) {
                            if (wb && lu[i].d + 1 > wb) { /* beyond this launch's window: later */
                                int32_t f = L[v];
                                for (int32_t q = 0; q < tmp_n[k]; ++q) if (lv[q].d <= lu[i].d + 1 && lv[q].v > f) f = lv[q].v;
                                if (lu[i].v > f) deferred[k] = 1;
                                continue;
                            }
                            r = ins(lv, &tmp_n[k], L[v], lu[i].d + 1, lu[i].v);
                            if (r < 0) { ++ovf; r = 0; }
                            changed |= r;
                        }
                    }
                    chg[k] = (uint8_t)changed;
                }
                for (long k = 0; k < m; ++k) {
                    if (!cur[k]) continue;
                    cur[k] = 0;
                    first[k] = 0;
                    if (!chg[k]) continue;
                    const int32_t v = tmem[a0 + k];
                    G2n[v] = tmp_n[k];
                    memcpy(&G2[(size_t)v * RMAX], &tmp_l[(size_t)k * RMAX], sizeof(ent_t) * (size_t)tmp_n[k]);
                    if (G2n[v] > maxlen) maxlen = G2n[v];
                    stamp[k] = levels;
                    for (int64_t e = rp[v]; e < rp[v + 1]; ++e) {
                        const int32_t u = col[e];
                        if (tile_of[u] == t) {
                            long lo = 0, hi = m;
                            while (lo < hi) { long md = (lo + hi) / 2; if (tmem[a0 + md] < u) lo = md + 1; else hi = md; }
                            if (!nxt[lo]) { nxt[lo] = 1; ++nn; }
                        } else {
                            __atomic_store_n(&mk2[u], 1, __ATOMIC_RELAXED);
                            __atomic_store_n(&tact2[tile_of[u]], 1, __ATOMIC_RELAXED);
                        }
                    }
                }
                uint8_t *tmp = cur; cur = nxt; nxt = tmp;
                nc = nn;
            }
            for (long k = 0; k < m; ++k)
                if (deferred[k]) {
                    __atomic_store_n(&mk2[tmem[a0 + k]], 1, __ATOMIC_RELAXED);
                    __atomic_store_n(&tact2[t], 1, __ATOMIC_RELAXED);
                }
            free(tmp_l); free(tmp_n); free(chg); free(stamp); free(first); free(deferred);
            lev_sum += levels;
            tlev[t] = (int32_t)levels;
            if (levels > launch_max) launch_max = levels;
            free(cur);
            free(nxt);
        }
        crit += launch_max;
        {   /* active tiles dealt round-robin (by rank) over kG workgroups: the launch lasts as long as
             * the workgroup with the most levels in sequence */
            long wl[kG] = {0}, wt[kG] = {0}, r = 0;
            for (long t = 0; t < ntiles; ++t)
                if (tact[t]) { wl[r % kG] += tlev[t]; wt[r % kG] += 1; ++r; }
            long ml = 0, mt = 0;
            for (int g = 0; g < kG; ++g) { if (wl[g] > ml) ml = wl[g]; if (wt[g] > mt) mt = wt[g]; }
            crit_wg += ml;
            crit_tiles += mt;
        }
        /* publish */
#pragma omp parallel for schedule(dynamic, 1)
        for (long t = 0; t < ntiles; ++t) {
            if (!tact[t]) continue;
            for (int64_t k = toff[t]; k < toff[t + 1]; ++k) {
                const int32_t v = tmem[k];
                Gn[v] = G2n[v];
                memcpy(&G[(size_t)v * RMAX], &G2[(size_t)v * RMAX], sizeof(ent_t) * (size_t)G2n[v]);
            }
        }
        for (long v = 0; v < n; ++v) { mk[v] |= mk2[v]; mk2[v] = 0; }
        memcpy(tact, tact2, (size_t)ntiles);
        memset(tact2, 0, (size_t)ntiles);
    }
    long dmax = 0;
    for (long v = 0; v < n; ++v) {
        int32_t b = L[v];
        for (int32_t i = 0; i < Gn[v]; ++i) {
            const ent_t e = G[(size_t)v * RMAX + i];
            if (e.d < hist_cap) hist[e.d] += 1;
            if (e.d > dmax) dmax = e.d;
            b = e.v;
        }
        final_leader[v] = b;
    }
    stats[0] = launches; stats[1] = acts; stats[2] = lev_sum; stats[3] = crit;
    stats[4] = maxlen; stats[5] = ovf; stats[6] = relax; stats[7] = edges;
    stats[8] = crit_wg; stats[9] = crit_tiles;
    free(tlev);
    free(G); free(Gn); free(G2); free(G2n); free(mk); free(mk2); free(tact); free(tact2);
    return dmax;
}
