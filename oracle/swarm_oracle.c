/*
 * swarm_oracle.c -- CPU restatement of the reference's per-round swarm step.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it.  The product path (libswarm.so) never links or
 * calls it.
 *
 * Parity is pinned: tests/test_oracle_golden.py checks every function below against the
 * golden vectors that tools/gen_golden.py produced by driving the reference's own handlers.
 *
 * Restated reference behaviour (file:line into the reference agent.py):
 *   orc_elect     _handle_election_acclaim (263-275) / _handle_heartbeat (243-261) under the
 *                 synchronous round contract E2:
 *                 leader'[v] = max(leader[v], max_{u in N(v)} leader[u]); state LEADER iff
 *                 leader == id; stop after the first round with zero changes.
 *   orc_utility   _calculate_utility (338-347): d = sqrt(pow(dx,2) + pow(dy,2)),
 *                 U = (100/(1+d)) * has_cap.  `**2` is CPython float_pow -> libm pow(x, 2.0),
 *                 so this file is compiled with -fno-builtin (gcc would fold pow(x,2) to x*x).
 *   orc_allocate  _process_tasks (292-302): claim iff U > 20.0 (fp64), payload f32(U) (RNE);
 *                 _handle_task_claim (304-325) at the single resolver in ascending sender
 *                 order: first claim wins, later claim wins iff x > u_cur + 5.0 (fp64);
 *                 every accepted claim and every rejected claim from a non-incumbent emits one
 *                 TASK_CONFLICT (322, 325).
 *   orc_rgg_csr   synthetic input builder (not reference code): edge iff dx*dx+dy*dy <= r*r.
 *   orc_auction   the north star's auction allocation (no reference code; see its comment).
 *   orc_physics   _update_physics (94-181) under the synchronous step contract P1.
 *   orc_protocol  the timer FSM (_check_election_timeout 217-241, _send_heartbeat 283-289) and
 *                 the election handlers (243-281) ticking under contract T1.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ST_FOLLOWER 1
#define ST_LEADER 3

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* Election to convergence.  leader[] is the working buffer (in: ignored, out: final).
 * changes[] receives per-round change counts (capacity max_rounds).  Returns rounds_exec,
 * or -1 if max_rounds passed without a zero-change round. */
long orc_elect(long n, const int64_t *row_ptr, const int32_t *col, const int32_t *ids,
               int32_t *leader, uint8_t *state, long max_rounds, int64_t *changes) {
    int32_t *next = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (long v = 0; v < n; ++v) leader[v] = ids[v];
    long rounds = 0, done = 0;
    while (rounds < max_rounds) {
        long c = 0;
#pragma omp parallel for schedule(static) reduction(+ : c)
        for (long v = 0; v < n; ++v) {
            int32_t m = leader[v];
            for (int64_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
                int32_t s = leader[col[e]];
                if (s > m) m = s;
            }
            next[v] = m;
            c += (m != leader[v]);
        }
        memcpy(leader, next, sizeof(int32_t) * (size_t)n);
        changes[rounds++] = c;
        if (c == 0) { done = 1; break; }
    }
    for (long v = 0; v < n; ++v) state[v] = (leader[v] == ids[v]) ? ST_LEADER : ST_FOLLOWER;
    free(next);
    return done ? rounds : -1;
}

/* Election to convergence, frontier form: the same rounds, leaders, rounds_exec and per-round
 * change counts as orc_elect, but round t+1 only recomputes the agents marked by round t's
 * risers -- each riser itself and every agent that hears it.  Exact: an unmarked agent's value
 * already dominates every neighbour value, none of which changed.  hear_ptr/hear_col is the
 * transpose of row_ptr/col (who hears v); pass NULL when the graph is symmetric.  Leaders are
 * double-buffered by round parity: the write buffer holds round t-2's state, which differs
 * from round t-1's only on round t-1's risers, all self-marked.  active[] (capacity max_rounds,
 * may be NULL) receives the agents recomputed per round.  Restates orc_elect (agent.py:243-275
 * under E2); it is pinned against orc_elect in tests/test_oracle_golden.py. */
long orc_elect_frontier(long n, const int64_t *row_ptr, const int32_t *col, const int64_t *hear_ptr,
                        const int32_t *hear_col, const int32_t *ids, int32_t *leader, uint8_t *state,
                        long max_rounds, int64_t *changes, int64_t *active) {
    const size_t nn = (size_t)(n > 0 ? n : 1);
    int32_t *buf[2];
    buf[0] = (int32_t *)malloc(sizeof(int32_t) * nn);
    buf[1] = (int32_t *)malloc(sizeof(int32_t) * nn);
    uint8_t *mark[2];
    mark[0] = (uint8_t *)calloc(nn, 1);
    mark[1] = (uint8_t *)malloc(nn);
    memset(mark[1], 1, nn); /* round 1 recomputes everyone */
    if (!hear_ptr) { hear_ptr = row_ptr; hear_col = col; }
    for (long v = 0; v < n; ++v) buf[0][v] = buf[1][v] = ids[v];
    long rounds = 0, done = 0;
    while (rounds < max_rounds) {
        const long t = rounds + 1;
        const int32_t *P = buf[(t - 1) & 1];
        int32_t *Q = buf[t & 1];
        uint8_t *cur = mark[t & 1], *nxt = mark[(t + 1) & 1];
        long c = 0, act = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : c, act)
        for (long v = 0; v < n; ++v) {
            if (!cur[v]) continue;
            cur[v] = 0;
            ++act;
            int32_t m = P[v];
            for (int64_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) {
                const int32_t s = P[col[e]];
                if (s > m) m = s;
            }
            Q[v] = m;
            if (m > P[v]) {
                ++c;
                __atomic_store_n(&nxt[v], (uint8_t)1, __ATOMIC_RELAXED);
                for (int64_t e = hear_ptr[v]; e < hear_ptr[v + 1]; ++e)
                    __atomic_store_n(&nxt[hear_col[e]], (uint8_t)1, __ATOMIC_RELAXED);
            }
        }
        changes[rounds] = c;
        if (active) active[rounds] = act;
        ++rounds;
        if (c == 0) { done = 1; break; }
    }
    const int32_t *fin = buf[rounds & 1];
    for (long v = 0; v < n; ++v) {
        leader[v] = fin[v];
        state[v] = (fin[v] == ids[v]) ? ST_LEADER : ST_FOLLOWER;
    }
    free(buf[0]); free(buf[1]); free(mark[0]); free(mark[1]);
    return done ? rounds : -1;
}

/* One utility, reference arithmetic (libm pow) or GPU arithmetic (x*x) by `use_pow`. */
static inline double util_one(double ax, double ay, uint32_t caps, double tx, double ty,
                              int8_t treq, double u_scale, int use_pow) {
    double dx = ax - tx, dy = ay - ty;
    double sx = use_pow ? pow(dx, 2.0) : dx * dx;
    double sy = use_pow ? pow(dy, 2.0) : dy * dy;
    double d = sqrt(sx + sy);
    /* agent.py:343-345: a required capability the agent lacks -> 0.0.  Indices >= 32 name a
     * capability outside the 32-bit mask, which no agent holds (no shift by >= 32: UB in C). */
    double has = (treq < 0) ? 1.0 : (treq < 32 && ((caps >> treq) & 1u)) ? 1.0 : 0.0;
    return (u_scale / (1.0 + d)) * has;
}

void orc_utility(long m, const double *ax, const double *ay, const uint32_t *caps,
                 const double *tx, const double *ty, const int8_t *treq, double u_scale,
                 int use_pow, double *out) {
#pragma omp parallel for schedule(static)
    for (long i = 0; i < m; ++i)
        out[i] = util_one(ax[i], ay[i], caps[i], tx[i], ty[i], treq[i], u_scale, use_pow);
}

static int cmp_by_id(const void *a, const void *b, void *ids) {
    int32_t x = ((const int32_t *)ids)[*(const long *)a], y = ((const int32_t *)ids)[*(const long *)b];
    return (x > y) - (x < y);
}

static const int32_t *g_ids;
static int cmp_by_id_g(const void *a, const void *b) { return cmp_by_id(a, b, (void *)g_ids); }

/* Dense allocation (every agent x every task).  winner[]/util[] are in/out chain state
 * (winner -1 = no current claim).  Per-task outputs: nclaim[k] claims, nmsg[k] conflict
 * messages.  won[] (per agent, storage order) counts final wins.  Returns total claims. */
long orc_allocate(long n, const int32_t *ids, const double *ax, const double *ay,
                  const uint32_t *caps, long t, const double *tx, const double *ty,
                  const int8_t *treq, double claim_thr, double hyst, double u_scale, int use_pow,
                  int32_t *winner, double *util, int64_t *nclaim, int64_t *nmsg, int32_t *won) {
    long *order = (long *)malloc(sizeof(long) * (size_t)(n > 0 ? n : 1));
    for (long i = 0; i < n; ++i) order[i] = i;
    g_ids = ids;
    qsort(order, (size_t)n, sizeof(long), cmp_by_id_g);
    long total = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : total)
    for (long k = 0; k < t; ++k) {
        int32_t w = winner[k];
        double u = util[k];
        int has = w >= 0;
        int64_t cl = 0, ms = 0;
        for (long j = 0; j < n; ++j) {
            long i = order[j];
            double U = util_one(ax[i], ay[i], caps[i], tx[k], ty[k], treq[k], u_scale, use_pow);
            if (!(U > claim_thr)) continue;
            ++cl;
            double x = (double)(float)U;
            if (!has || x > u + hyst) {
                w = ids[i]; u = x; has = 1; ++ms;
            } else if (w != ids[i]) {
                ++ms;
            }
        }
        winner[k] = w; util[k] = u; nclaim[k] = cl; nmsg[k] = ms; total += cl;
    }
    for (long i = 0; i < n; ++i) won[i] = 0;
    /* won: map winner id -> storage index via the sorted order (binary search) */
    for (long k = 0; k < t; ++k) {
        if (winner[k] < 0) continue;
        long lo = 0, hi = n - 1;
        while (lo <= hi) {
            long mid = (lo + hi) / 2;
            int32_t v = ids[order[mid]];
            if (v == winner[k]) { won[order[mid]] += 1; break; }
            if (v < winner[k]) lo = mid + 1; else hi = mid - 1;
        }
    }
    free(order);
    return total;
}

/* orc_allocate restricted to the agents that can claim: with claim_thr > 0 and u_scale > 0 a
 * claim needs U > claim_thr, i.e. d < u_scale / claim_thr - 1, so only agents inside that radius
 * (widened by a relative 1e-9 against rounding) are evaluated, found through a uniform grid.
 * Same outputs as orc_allocate (pinned against it in tests/test_oracle_golden.py); falls back to
 * it when the claim radius is not finite.  The CPU baseline of the GPU's binned allocation. */
typedef struct { int32_t id; float x; long idx; } claim_t;
static int cmp_claim(const void *a, const void *b) {
    const claim_t *p = (const claim_t *)a, *q = (const claim_t *)b;
    return (p->id > q->id) - (p->id < q->id);
}

long orc_allocate_binned(long n, const int32_t *ids, const double *ax, const double *ay,
                         const uint32_t *caps, long t, const double *tx, const double *ty,
                         const int8_t *treq, double claim_thr, double hyst, double u_scale, int use_pow,
                         int32_t *winner, double *util, int64_t *nclaim, int64_t *nmsg, int32_t *won) {
    if (!(claim_thr > 0 && u_scale > 0) || n == 0)
        return orc_allocate(n, ids, ax, ay, caps, t, tx, ty, treq, claim_thr, hyst, u_scale, use_pow, winner,
                            util, nclaim, nmsg, won);
    /* rp <= 0: nobody can claim, every task keeps its current claim (the loop finds no claims) */
    const double rp = (u_scale / claim_thr - 1.0) * (1.0 + 1e-9) + 1e-12;
    double xmin = ax[0], xmax = ax[0], ymin = ay[0], ymax = ay[0];
    for (long i = 1; i < n; ++i) {
        if (ax[i] < xmin) xmin = ax[i];
        if (ax[i] > xmax) xmax = ax[i];
        if (ay[i] < ymin) ymin = ay[i];
        if (ay[i] > ymax) ymax = ay[i];
    }
    double cell = rp > 0 ? rp : 1.0;
    long ncx, ncy;
    for (;;) {
        ncx = (long)floor((xmax - xmin) / cell) + 1;
        ncy = (long)floor((ymax - ymin) / cell) + 1;
        if ((double)ncx * (double)ncy <= 2.0 * (double)n + 1024.0) break;
        cell *= 1.4142135623730951;
    }
    long *start = (long *)calloc((size_t)(ncx * ncy + 1), sizeof(long));
    long *cellof = (long *)malloc(sizeof(long) * (size_t)n);
    for (long i = 0; i < n; ++i) {
        long cx = (long)floor((ax[i] - xmin) / cell), cy = (long)floor((ay[i] - ymin) / cell);
        cx = cx < 0 ? 0 : cx >= ncx ? ncx - 1 : cx;
        cy = cy < 0 ? 0 : cy >= ncy ? ncy - 1 : cy;
        cellof[i] = cy * ncx + cx;
        start[cellof[i] + 1]++;
    }
    for (long c = 0; c < ncx * ncy; ++c) start[c + 1] += start[c];
    long *fillp = (long *)malloc(sizeof(long) * (size_t)(ncx * ncy));
    for (long c = 0; c < ncx * ncy; ++c) fillp[c] = start[c];
    long *members = (long *)malloc(sizeof(long) * (size_t)n);
    for (long i = 0; i < n; ++i) members[fillp[cellof[i]]++] = i;
    /* id -> storage index (won credit for a pre-existing winner that keeps its task) */
    long *order = (long *)malloc(sizeof(long) * (size_t)n);
    for (long i = 0; i < n; ++i) order[i] = i;
    g_ids = ids;
    qsort(order, (size_t)n, sizeof(long), cmp_by_id_g);
    long total = 0;
#pragma omp parallel reduction(+ : total)
    {
        long cap = 1024;
        claim_t *cl = (claim_t *)malloc(sizeof(claim_t) * (size_t)cap);
#pragma omp for schedule(dynamic, 16)
        for (long k = 0; k < t; ++k) {
            long m = 0;
            if (rp > 0) {
                long x0 = (long)floor((tx[k] - rp - xmin) / cell), x1 = (long)floor((tx[k] + rp - xmin) / cell);
                long y0 = (long)floor((ty[k] - rp - ymin) / cell), y1 = (long)floor((ty[k] + rp - ymin) / cell);
                x0 = x0 < 0 ? 0 : x0; y0 = y0 < 0 ? 0 : y0;
                x1 = x1 >= ncx ? ncx - 1 : x1; y1 = y1 >= ncy ? ncy - 1 : y1;
                for (long cy = y0; cy <= y1; ++cy)
                    for (long cx = x0; cx <= x1; ++cx)
                        for (long p = start[cy * ncx + cx]; p < start[cy * ncx + cx + 1]; ++p) {
                            const long i = members[p];
                            const double U = util_one(ax[i], ay[i], caps[i], tx[k], ty[k], treq[k], u_scale, use_pow);
                            if (!(U > claim_thr)) continue;
                            if (m == cap) {
                                cap *= 2;
                                cl = (claim_t *)realloc(cl, sizeof(claim_t) * (size_t)cap);
                            }
                            cl[m].id = ids[i];
                            cl[m].x = (float)U;
                            cl[m].idx = i;
                            ++m;
                        }
            }
            qsort(cl, (size_t)m, sizeof(claim_t), cmp_claim);
            int32_t w = winner[k];
            double u = util[k];
            int has = w >= 0;
            int64_t ms = 0;
            for (long j = 0; j < m; ++j) {
                const double x = (double)cl[j].x;
                if (!has || x > u + hyst) {
                    w = cl[j].id; u = x; has = 1; ++ms;
                } else if (w != cl[j].id) {
                    ++ms;
                }
            }
            winner[k] = w; util[k] = u; nclaim[k] = m; nmsg[k] = ms; total += m;
        }
        free(cl);
    }
    for (long i = 0; i < n; ++i) won[i] = 0;
    for (long k = 0; k < t; ++k) {
        if (winner[k] < 0) continue;
        long lo = 0, hi = n - 1;
        while (lo <= hi) {
            long mid = (lo + hi) / 2;
            int32_t v = ids[order[mid]];
            if (v == winner[k]) { won[order[mid]] += 1; break; }
            if (v < winner[k]) lo = mid + 1; else hi = mid - 1;
        }
    }
    free(start); free(cellof); free(fillp); free(members); free(order);
    return total;
}

/* Claims of one task only, in ascending-ID order (for chain-kernel debugging and the
 * argmax comparisons in tests).  Returns the number written (<= cap). */
long orc_task_claims(long n, const int32_t *ids, const double *ax, const double *ay,
                     const uint32_t *caps, double tx, double ty, int8_t treq, double claim_thr,
                     double u_scale, int use_pow, int32_t *out_id, float *out_x, long cap) {
    long *order = (long *)malloc(sizeof(long) * (size_t)(n > 0 ? n : 1));
    for (long i = 0; i < n; ++i) order[i] = i;
    g_ids = ids;
    qsort(order, (size_t)n, sizeof(long), cmp_by_id_g);
    long m = 0;
    for (long j = 0; j < n; ++j) {
        long i = order[j];
        double U = util_one(ax[i], ay[i], caps[i], tx, ty, treq, u_scale, use_pow);
        if (U > claim_thr) {
            if (m < cap) { out_id[m] = ids[i]; out_x[m] = (float)U; }
            ++m;
        }
    }
    free(order);
    return m;
}

/* Radius-r geometric graph, rows sorted ascending.  Two calls: row_ptr only (col == NULL)
 * to size, then fill.  Cell list with cells of side r. */
typedef struct { long key; long idx; } kv_t;
static int cmp_kv(const void *a, const void *b) {
    const kv_t *x = (const kv_t *)a, *y = (const kv_t *)b;
    if (x->key != y->key) return (x->key > y->key) - (x->key < y->key);
    return (x->idx > y->idx) - (x->idx < y->idx);
}
static int cmp_i32(const void *a, const void *b) {
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

long orc_rgg_csr(long n, const double *x, const double *y, double r, int64_t *row_ptr,
                 int32_t *col) {
    if (n == 0) { row_ptr[0] = 0; return 0; }
    double r2 = r * r;
    long maxcx = 0, maxcy = 0;
    for (long i = 0; i < n; ++i) {
        long cx = (long)floor(x[i] / r), cy = (long)floor(y[i] / r);
        if (cx > maxcx) maxcx = cx;
        if (cy > maxcy) maxcy = cy;
    }
    long ncx = maxcx + 3, ncy = maxcy + 3;
    kv_t *kv = (kv_t *)malloc(sizeof(kv_t) * (size_t)n);
    for (long i = 0; i < n; ++i) {
        long cx = (long)floor(x[i] / r), cy = (long)floor(y[i] / r);
        kv[i].key = (cy + 1) * ncx + (cx + 1);
        kv[i].idx = i;
    }
    qsort(kv, (size_t)n, sizeof(kv_t), cmp_kv);
    long ncell = ncx * ncy;
    long *start = (long *)calloc((size_t)ncell + 1, sizeof(long));
    for (long i = 0; i < n; ++i) start[kv[i].key + 1]++;
    for (long c = 0; c < ncell; ++c) start[c + 1] += start[c];
    int fill = col != NULL;
    if (!fill) row_ptr[0] = 0;
#pragma omp parallel for schedule(dynamic, 1024)
    for (long i = 0; i < n; ++i) {
        long cx = (long)floor(x[i] / r) + 1, cy = (long)floor(y[i] / r) + 1;
        long cnt = 0;
        int64_t base = fill ? row_ptr[i] : 0;
        for (long oy = -1; oy <= 1; ++oy)
            for (long ox = -1; ox <= 1; ++ox) {
                long c = (cy + oy) * ncx + (cx + ox);
                for (long p = start[c]; p < start[c + 1]; ++p) {
                    long j = kv[p].idx;
                    if (j == i) continue;
                    double dx = x[i] - x[j], dy = y[i] - y[j];
                    if (dx * dx + dy * dy <= r2) {
                        if (fill) col[base + cnt] = (int32_t)j;
                        ++cnt;
                    }
                }
            }
        if (fill) qsort(col + base, (size_t)cnt, sizeof(int32_t), cmp_i32);
        else row_ptr[i + 1] = cnt;
    }
    if (!fill)
        for (long i = 0; i < n; ++i) row_ptr[i + 1] += row_ptr[i];
    free(start);
    free(kv);
    return (long)row_ptr[n];
}

/* ------------------------------------------------------------------ auction
 * No reference counterpart: the north star's "auction price update" allocation, restated here
 * as the checker of the GPU bid/resolve kernels (parity vs this restatement only).
 * Jacobi (synchronous) Bertsekas auction over the admissible pairs U > claim_thr -- the
 * reference's claim rule (agent.py:297) -- with value x = f32(U), the claim payload
 * (agent.py:302).  Per round every unassigned, active agent a finds, over its admissible
 * tasks, net = x - price[k] (f32), the best (ties -> lowest task index) and second-best net,
 * with the opt-out option (net 0) as a competitor: best <= 0 -> a drops out for good (prices
 * only rise); else it bids price[best] + (best - second) + eps (f32, in that order).  Each task
 * takes its highest bid, ties -> lowest agent ID (packed key: f32 bits << 32 | ~id), the
 * previous owner becomes unassigned.  Stops after the first round without bidders;
 * rounds_exec = rounds that had bidders.  assigned[a] = task index or -1; owner[k] = agent
 * storage index or -1; bidders[r] = active agents of round r+1. */
static uint32_t f32_bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static float bits_f32(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* Uniform grid over task positions (cells of side >= r, at most 2t + 1024 cells); members of a
 * cell in ascending task index. */
typedef struct { double xmin, ymin, cell, r; long ncx, ncy; long *start, *members; } task_grid_t;

static void task_grid_build(task_grid_t *g, long t, const double *tx, const double *ty, double r) {
    double xmin = tx[0], xmax = tx[0], ymin = ty[0], ymax = ty[0];
    for (long k = 1; k < t; ++k) {
        if (tx[k] < xmin) xmin = tx[k];
        if (tx[k] > xmax) xmax = tx[k];
        if (ty[k] < ymin) ymin = ty[k];
        if (ty[k] > ymax) ymax = ty[k];
    }
    double cell = r > 0 ? r : 1.0;
    for (;;) {
        g->ncx = (long)floor((xmax - xmin) / cell) + 1;
        g->ncy = (long)floor((ymax - ymin) / cell) + 1;
        if ((double)g->ncx * (double)g->ncy <= 2.0 * (double)t + 1024.0) break;
        cell *= 1.4142135623730951;
    }
    g->xmin = xmin; g->ymin = ymin; g->cell = cell; g->r = r;
    const long nc = g->ncx * g->ncy;
    g->start = (long *)calloc((size_t)nc + 1, sizeof(long));
    g->members = (long *)malloc(sizeof(long) * (size_t)t);
    long *cof = (long *)malloc(sizeof(long) * (size_t)t);
    for (long k = 0; k < t; ++k) {
        long cx = (long)floor((tx[k] - xmin) / cell), cy = (long)floor((ty[k] - ymin) / cell);
        cx = cx < 0 ? 0 : cx >= g->ncx ? g->ncx - 1 : cx;
        cy = cy < 0 ? 0 : cy >= g->ncy ? g->ncy - 1 : cy;
        cof[k] = cy * g->ncx + cx;
        g->start[cof[k] + 1]++;
    }
    for (long c = 0; c < nc; ++c) g->start[c + 1] += g->start[c];
    long *fp = (long *)malloc(sizeof(long) * (size_t)(nc > 0 ? nc : 1));
    for (long c = 0; c < nc; ++c) fp[c] = g->start[c];
    for (long k = 0; k < t; ++k) g->members[fp[cof[k]]++] = k;  /* ascending k within a cell */
    free(fp);
    free(cof);
}

static void task_grid_free(task_grid_t *g) { free(g->start); free(g->members); }

static int cmp_ck(const void *a, const void *b) {
    const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

/* Admissible tasks (U > thr) of one agent; with out_k/out_v, written in ascending task index
 * (values follow their tasks).  Returns the count. */
static int64_t task_grid_claims(const task_grid_t *g, double px, double py, uint32_t cap, const double *tx,
                                const double *ty, const int8_t *treq, double thr, double u_scale, int use_pow,
                                int32_t *out_k, float *out_v) {
    if (!(g->r > 0)) return 0;
    long x0 = (long)floor((px - g->r - g->xmin) / g->cell), x1 = (long)floor((px + g->r - g->xmin) / g->cell);
    long y0 = (long)floor((py - g->r - g->ymin) / g->cell), y1 = (long)floor((py + g->r - g->ymin) / g->cell);
    x0 = x0 < 0 ? 0 : x0; y0 = y0 < 0 ? 0 : y0;
    x1 = x1 >= g->ncx ? g->ncx - 1 : x1; y1 = y1 >= g->ncy ? g->ncy - 1 : y1;
    int64_t c = 0;
    for (long cy = y0; cy <= y1; ++cy)
        for (long cx = x0; cx <= x1; ++cx)
            for (long p = g->start[cy * g->ncx + cx]; p < g->start[cy * g->ncx + cx + 1]; ++p) {
                const long k = g->members[p];
                if (util_one(px, py, cap, tx[k], ty[k], treq[k], u_scale, use_pow) > thr) {
                    if (out_k) out_k[c] = (int32_t)k;
                    ++c;
                }
            }
    if (out_k) {
        qsort(out_k, (size_t)c, sizeof(int32_t), cmp_ck);
        for (int64_t j = 0; j < c; ++j)
            out_v[j] = (float)util_one(px, py, cap, tx[out_k[j]], ty[out_k[j]], treq[out_k[j]], u_scale, use_pow);
    }
    return c;
}

long orc_auction(long n, const int32_t *ids, const double *ax, const double *ay, const uint32_t *caps,
                 long t, const double *tx, const double *ty, const int8_t *treq, double claim_thr,
                 double u_scale, int use_pow, float eps, long max_rounds, int32_t *owner, float *price,
                 int32_t *assigned, int64_t *bidders, int64_t *n_pairs) {
    int64_t *off = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    /* candidate tasks of each agent in ascending task index: through a uniform grid over the
     * tasks when the claim radius is finite (U > thr needs d < u_scale/thr - 1), else all */
    task_grid_t tg;
    const int binned = claim_thr > 0 && u_scale > 0 && t > 0;
    if (binned) task_grid_build(&tg, t, tx, ty, (u_scale / claim_thr - 1.0) * (1.0 + 1e-9) + 1e-12);
#pragma omp parallel for schedule(dynamic, 64)
    for (long a = 0; a < n; ++a) {
        int64_t c = 0;
        if (binned) {
            c = task_grid_claims(&tg, ax[a], ay[a], caps[a], tx, ty, treq, claim_thr, u_scale, use_pow, NULL, NULL);
        } else {
            for (long k = 0; k < t; ++k)
                if (util_one(ax[a], ay[a], caps[a], tx[k], ty[k], treq[k], u_scale, use_pow) > claim_thr) ++c;
        }
        off[a + 1] = c;
    }
    for (long a = 0; a < n; ++a) off[a + 1] += off[a];
    const int64_t np = off[n];
    int32_t *ck = (int32_t *)malloc(sizeof(int32_t) * (size_t)(np > 0 ? np : 1));
    float *cv = (float *)malloc(sizeof(float) * (size_t)(np > 0 ? np : 1));
#pragma omp parallel for schedule(dynamic, 64)
    for (long a = 0; a < n; ++a) {
        int64_t p = off[a];
        if (binned) {
            task_grid_claims(&tg, ax[a], ay[a], caps[a], tx, ty, treq, claim_thr, u_scale, use_pow, ck + p, cv + p);
            continue;
        }
        for (long k = 0; k < t; ++k) {
            double U = util_one(ax[a], ay[a], caps[a], tx[k], ty[k], treq[k], u_scale, use_pow);
            if (U > claim_thr) { ck[p] = (int32_t)k; cv[p] = (float)U; ++p; }
        }
    }
    if (binned) task_grid_free(&tg);
    if (n_pairs) *n_pairs = np;
    /* id -> storage index via the ascending-ID order */
    long *order = (long *)malloc(sizeof(long) * (size_t)(n > 0 ? n : 1));
    for (long i = 0; i < n; ++i) order[i] = i;
    g_ids = ids;
    qsort(order, (size_t)n, sizeof(long), cmp_by_id_g);
    uint8_t *out = (uint8_t *)calloc((size_t)n + 1, 1);
    uint64_t *key = (uint64_t *)calloc((size_t)t + 1, sizeof(uint64_t));
    for (long k = 0; k < t; ++k) { owner[k] = -1; price[k] = 0.0f; }
    for (long a = 0; a < n; ++a) assigned[a] = -1;
    long r = 0, done = 0;
    while (r < max_rounds) {
        int64_t nb = 0;
        for (long a = 0; a < n; ++a) {
            if (assigned[a] >= 0 || out[a]) continue;
            ++nb;
            float best = -INFINITY, second = -INFINITY;
            int32_t bk = INT32_MAX;
            for (int64_t p = off[a]; p < off[a + 1]; ++p) {
                const float net = cv[p] - price[ck[p]];
                if (net > best || (net == best && ck[p] < bk)) {
                    second = best > second ? best : second;
                    best = net;
                    bk = ck[p];
                } else if (net > second) {
                    second = net;
                }
            }
            if (!(best > 0.0f)) { out[a] = 1; continue; }
            if (second < 0.0f) second = 0.0f;
            const float inc = best - second;
            float bid = price[bk] + inc;
            bid = bid + eps;
            const uint64_t kk = ((uint64_t)f32_bits(bid) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)ids[a]);
            if (kk > key[bk]) key[bk] = kk;
        }
        if (nb == 0) { done = 1; break; }
        if (bidders) bidders[r] = nb;
        ++r;
        for (long k = 0; k < t; ++k) {
            if (!key[k]) continue;
            const int32_t wid = (int32_t)(0xFFFFFFFFu - (uint32_t)(key[k] & 0xFFFFFFFFu));
            long lo = 0, hi = n - 1, w = -1;
            while (lo <= hi) {
                const long mid = (lo + hi) / 2;
                const int32_t v = ids[order[mid]];
                if (v == wid) { w = order[mid]; break; }
                if (v < wid) lo = mid + 1; else hi = mid - 1;
            }
            if (owner[k] >= 0) assigned[owner[k]] = -1;
            owner[k] = (int32_t)w;
            assigned[w] = (int32_t)k;
            price[k] = bits_f32((uint32_t)(key[k] >> 32));
            key[k] = 0;
        }
    }
    free(off); free(ck); free(cv); free(order); free(out); free(key);
    return done ? r : -1;
}

/* ------------------------------------------------------------------ physics
 * _update_physics (agent.py:94-181) under the synchronous step contract P1 (tools/gen_golden.py):
 * every agent reads the step-start snapshot of all positions; a FOLLOWER with a leader targets
 * the V-formation slot behind the f32-rounded leader position (the '!ff' heartbeat payload,
 * agent.py:256-258, 283-289): x - 2 id, y + 2 id (even id) or y - 2 id (odd id) (agent.py:96-111);
 * no target -> no motion (113-114).  Forces (fp64, the reference's order of operations):
 * attraction (target - p) if |target - p| > 0.5 (118-125); obstacles in list order, d = |p - o| - r
 * clamped to 0.001, if d < 5: 50 (1/d - 1/5) / d^2 along (p - o)/|p - o| (128-146); neighbours
 * in CSR order, d = |p - q|, if d < 2: clamped, 20 / d^2 along (p - q)/|p - q| (149-160); speed
 * clamp to max_speed (169-174); Euler step (177-178).  `**2` is libm pow (use_pow) or x*x.
 * A zero |p - o| or |p - q| makes the reference raise ZeroDivisionError; here it yields
 * non-finite values and is counted (return value). */
long orc_physics(long n, const int32_t *ids, const uint8_t *state, const int32_t *leader, double *x, double *y,
                 double *vx, double *vy, double *tx, double *ty, uint8_t *has_t, long m, const double *obs,
                 const int64_t *row_ptr, const int32_t *col, double dt, double max_speed, long steps,
                 int use_pow) {
    double *sx = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *sy = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    long singular = 0;
#define SQ(v) (use_pow ? pow((v), 2.0) : (v) * (v))
    for (long st = 0; st < steps; ++st) {
        memcpy(sx, x, sizeof(double) * (size_t)n);
        memcpy(sy, y, sizeof(double) * (size_t)n);
#pragma omp parallel for schedule(static) reduction(+ : singular)
        for (long i = 0; i < n; ++i) {
            const double px = sx[i], py = sy[i];
            if (state[i] == ST_FOLLOWER && leader[i] >= 0) {
                const double lx = (double)(float)sx[leader[i]], ly = (double)(float)sy[leader[i]];
                const double rank = (double)ids[i];
                const double xo = -2.0 * rank;
                const double yo = (ids[i] % 2 == 0) ? 2.0 * rank : -2.0 * rank;
                tx[i] = lx + xo;
                ty[i] = ly + yo;
                has_t[i] = 1;
            }
            if (!has_t[i]) continue;
            double fax = 0.0, fay = 0.0;
            const double dtg = sqrt(SQ(tx[i] - px) + SQ(ty[i] - py));
            if (dtg > 0.5) {
                fax = 1.0 * (tx[i] - px);
                fay = 1.0 * (ty[i] - py);
            }
            double frx = 0.0, fry = 0.0;
            for (long o = 0; o < m; ++o) {
                const double ox = obs[3 * o], oy = obs[3 * o + 1], r = obs[3 * o + 2];
                double d = sqrt(SQ(px - ox) + SQ(py - oy)) - r;
                if (d <= 0.001) d = 0.001;
                if (d < 5.0) {
                    const double mag = 50.0 * (1.0 / d - 1.0 / 5.0) / SQ(d);
                    const double dx = px - ox, dy = py - oy;
                    const double nrm = sqrt(SQ(dx) + SQ(dy));
                    if (nrm == 0.0) ++singular;
                    frx += (dx / nrm) * mag;
                    fry += (dy / nrm) * mag;
                }
            }
            double fsx = 0.0, fsy = 0.0;
            for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
                const long j = col[k];
                const double qx = sx[j], qy = sy[j];
                double d = sqrt(SQ(px - qx) + SQ(py - qy));
                if (d < 2.0) {
                    if (d <= 0.001) d = 0.001;
                    const double mag = 20.0 / SQ(d);
                    const double dx = px - qx, dy = py - qy;
                    const double nrm = sqrt(SQ(dx) + SQ(dy));
                    if (nrm == 0.0) ++singular;
                    fsx += (dx / nrm) * mag;
                    fsy += (dy / nrm) * mag;
                }
            }
            const double f0 = fax + frx + fsx, f1 = fay + fry + fsy;
            const double vmag = sqrt(SQ(f0) + SQ(f1));
            if (vmag > max_speed) {
                const double scale = max_speed / vmag;
                vx[i] = f0 * scale;
                vy[i] = f1 * scale;
            } else {
                vx[i] = f0;
                vy[i] = f1;
            }
            x[i] = px + vx[i] * dt;
            y[i] = py + vy[i] * dt;
        }
    }
#undef SQ
    free(sx);
    free(sy);
    return singular;
}


/* ---------------------------------------------------------------------- timer FSM (T1) */
#define ST_WAIT 2
#define OB_ACCLAIM 1u /* ELECTION_ACCLAIM followed by COORDINATOR (agent.py:240-241) */
#define OB_HB 2u      /* HEARTBEAT (289) */

/* random.uniform(0, 0.2)'s u: splitmix64 finaliser of (seed, id, tick), 53 high bits
 * (tools/gen_golden.py jitter_u). */
static double jitter_u(uint64_t seed, int32_t id, int64_t t) {
    uint64_t x = seed ^ ((uint64_t)(uint32_t)id * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)t * 0xD1B54A32D192ED03ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (double)(x >> 11) * (1.0 / 9007199254740992.0);
}

/* Ticks t = t0+1 .. t0+ticks of contract T1 (tools/gen_golden.py ref_fsm).  At tick t (clock
 * now = t*dt; agent i's own tick counter t + tick_off[i]):
 *   kills      if t is in kill_ticks, every alive LEADER dies (stops receiving and sending)
 *   receive    each alive agent handles what its CSR neighbours sent during tick t-1, in CSR
 *              order; one sender's packets within a tick are ACCLAIM, COORDINATOR, HEARTBEAT or
 *              just HEARTBEAT(s) -- a bully HEARTBEAT (249-251, 272-275) needs state LEADER,
 *              which rules out an ACCLAIM in the same tick, and a repeated HEARTBEAT is
 *              idempotent -- so a two-bit outbox carries them exactly:
 *                ACCLAIM (263-275): higher sender -> FOLLOWER, leader, liveness;
 *                  lower sender while LEADER / ELECTION_WAIT -> LEADER, bully heartbeat
 *                COORDINATOR (277-281): unconditional takeover
 *                HEARTBEAT (243-261): LEADER hearing a lower sender bullies back and stops;
 *                  else yield if LEADER, follow, liveness, leader_pos = f32 sender position,
 *                  ELECTION_WAIT -> FOLLOWER
 *              a heartbeat is sent only when the agent's own tick % 10 == 0 (288)
 *   logic      _check_election_timeout (217-241) then the LEADER's _send_heartbeat.
 * outbox: 2n bytes, tick parity double buffer (in: the tick-t0 outbox at parity t0&1).
 * counts (ticks x 4): alive LEADERs, alive ELECTION_WAITs, ACCLAIM senders, HEARTBEAT senders. */
void orc_protocol(long n, const int32_t *ids, const double *x, const double *y, const int64_t *row_ptr,
                  const int32_t *col, const int32_t *tick_off, uint8_t *state, int32_t *leader, double *last_hb,
                  double *wait_start, double *delay, float *lpos, uint8_t *has_lpos, uint8_t *alive,
                  uint8_t *outbox, long t0, long ticks, double dt, double timeout, double jitter, uint64_t seed,
                  const int64_t *kill_ticks, long n_kill, int64_t *counts) {
    for (long t = t0 + 1; t <= t0 + ticks; ++t) {
        const double now = (double)t * dt;
        const uint8_t *ob_in = outbox + (size_t)((t - 1) & 1) * (size_t)n;
        uint8_t *ob_out = outbox + (size_t)(t & 1) * (size_t)n;
        int kill = 0;
        for (long k = 0; k < n_kill; ++k) kill |= kill_ticks[k] == t;
        int64_t *cnt = counts + 4 * (t - t0 - 1);
        cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
        for (long i = 0; i < n; ++i)
            if (kill && alive[i] && state[i] == ST_LEADER) alive[i] = 0;
        for (long i = 0; i < n; ++i) {
            uint8_t ob = 0;
            if (!alive[i]) {
                ob_out[i] = 0;
                continue;
            }
            const int32_t me = ids[i];
            const int hb_tick = ((t + tick_off[i]) % 10) == 0;
            uint8_t st = state[i];
            for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
                const int32_t j = col[k];
                const uint8_t o = ob_in[j];
                const int32_t s = ids[j];
                if (o & OB_ACCLAIM) {
                    if (s > me) {
                        st = ST_FOLLOWER;
                        leader[i] = s;
                        last_hb[i] = now;
                    } else if (s < me && (st == ST_LEADER || st == ST_WAIT)) {
                        if (st == ST_WAIT) {
                            st = ST_LEADER;
                            leader[i] = me;
                        }
                        if (hb_tick) ob |= OB_HB;
                    }
                    leader[i] = s; /* COORDINATOR */
                    st = ST_FOLLOWER;
                    last_hb[i] = now;
                }
                if (o & OB_HB) {
                    if (st == ST_LEADER && s < me) {
                        if (hb_tick) ob |= OB_HB;
                    } else {
                        if (st == ST_LEADER && s > me) st = ST_FOLLOWER;
                        leader[i] = s;
                        last_hb[i] = now;
                        lpos[2 * i] = (float)x[j];
                        lpos[2 * i + 1] = (float)y[j];
                        has_lpos[i] = 1;
                        if (st == ST_WAIT) st = ST_FOLLOWER;
                    }
                }
            }
            if (st != ST_LEADER) {
                if (st == ST_FOLLOWER && now - last_hb[i] > timeout) {
                    st = ST_WAIT;
                    wait_start[i] = now;
                    delay[i] = 0.0 + jitter * jitter_u(seed, me, t);
                    leader[i] = -1;
                    has_lpos[i] = 0; /* leader_pos = None: stored as (0, 0) */
                    lpos[2 * i] = lpos[2 * i + 1] = 0.0f;
                }
                if (st == ST_WAIT && now - wait_start[i] > delay[i]) {
                    st = ST_LEADER;
                    leader[i] = me;
                    ob |= OB_ACCLAIM;
                }
            }
            if (st == ST_LEADER && hb_tick) ob |= OB_HB;
            state[i] = st;
            ob_out[i] = ob;
        }
        for (long i = 0; i < n; ++i) {
            cnt[0] += alive[i] && state[i] == ST_LEADER;
            cnt[1] += alive[i] && state[i] == ST_WAIT;
            cnt[2] += (ob_out[i] & OB_ACCLAIM) != 0;
            cnt[3] += (ob_out[i] & OB_HB) != 0;
        }
    }
}
