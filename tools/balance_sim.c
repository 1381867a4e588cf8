/* CPU replay of the 10M-agent frontier election that prices static chunk -> workgroup rebalancing
 *  before building it.  Per sparse round: the marked agents per 2 048-slot chunk in
 * the interleaved stamp layout (32-agent blocks, block b -> chunk b % M; agent order once the previous
 * round changed < il_min agents), then two schedules of the chunks over NG workgroups:
 *   grid    chunk c -> workgroup c % NG (today's k_sparse_block)
 *   static  contiguous chunk ranges of equal predicted work, predicted from the PREVIOUS round's counts
 * with a per-workgroup time a + b * ceil(listed / 64) (one 64-agent gather pass per 4 waves), the round
 * taking its slowest workgroup.  Output: per round  t marked grid_max static_max ideal.
 * Build: gcc -O2 -fopenmp -shared -fPIC -o tools/libbalance_sim.so tools/balance_sim.c  (tools/balance_sim.py) */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int64_t slot_of(int64_t v, int64_t M, int interleaved) {
    if (!interleaved) return v;  /* agent order: chunk = v / 2048 */
    const int64_t b = v >> 5, c = b % M, k = b / M;
    return c * 2048 + k * 32 + (v & 31);
}

/* returns rounds; out[r * 4 + {0..3}] = marked, grid max listed, static max listed, ideal (mean) listed */
long balance_sim(long n, const int64_t *rp, const int32_t *col, const int32_t *ids, long NG, long il_min,
                 long max_rounds, int64_t *out) {
    int32_t *L = malloc(sizeof(int32_t) * n), *L2 = malloc(sizeof(int32_t) * n);
    uint8_t *mark = calloc(n, 1), *mark2 = calloc(n, 1);
    const int64_t M = (n + 2047) / 2048;
    int64_t *cnt = calloc(M, 8), *prev = calloc(M, 8), *cut = malloc(8 * (NG + 1));
    memcpy(L, ids, sizeof(int32_t) * n);
    long t, last_changes = n;
    for (int64_t v = 0; v < n; ++v) mark[v] = 1; /* round 1: everyone */
    for (t = 1; t <= max_rounds; ++t) {
        const int inter = last_changes >= il_min;
        memset(cnt, 0, 8 * M);
        int64_t marked = 0, changes = 0;
        memcpy(L2, L, sizeof(int32_t) * n);
        for (int64_t v = 0; v < n; ++v) {
            if (!mark[v]) continue;
            ++marked;
            cnt[slot_of(v, M, inter) >> 11]++;
            int32_t m = L[v];
            for (int64_t k = rp[v]; k < rp[v + 1]; ++k) if (L[col[k]] > m) m = L[col[k]];
            if (m > L[v]) L2[v] = m;
        }
        memset(mark2, 0, n);
        for (int64_t v = 0; v < n; ++v) {
            if (L2[v] == L[v]) continue;
            ++changes;
            mark2[v] = 1;
            for (int64_t k = rp[v]; k < rp[v + 1]; ++k) mark2[col[k]] = 1;
        }
        /* grid stride */
        int64_t gmax = 0;
        for (int64_t w = 0; w < NG; ++w) {
            int64_t s = 0;
            for (int64_t c = w; c < M; c += NG) s += cnt[c];
            if (s > gmax) gmax = s;
        }
        /* static: cuts from the previous round's counts (work = count + a chunk's fixed share) */
        int64_t tot = 0;
        for (int64_t c = 0; c < M; ++c) tot += prev[c] + 16;
        int64_t acc = 0, w = 0;
        cut[0] = 0;
        for (int64_t c = 0; c < M && w < NG - 1; ++c) {
            acc += prev[c] + 16;
            while (w < NG - 1 && acc * NG >= (w + 1) * tot) cut[++w] = c + 1;
        }
        while (w < NG) cut[++w] = M;
        int64_t smax = 0;
        for (int64_t q = 0; q < NG; ++q) {
            int64_t s = 0;
            for (int64_t c = cut[q]; c < cut[q + 1]; ++c) s += cnt[c];
            if (s > smax) smax = s;
        }
        memcpy(prev, cnt, 8 * M);
        out[t * 4 - 4] = marked;
        out[t * 4 - 3] = gmax;
        out[t * 4 - 2] = smax;
        out[t * 4 - 1] = (marked + NG - 1) / NG;
        int32_t *tmp = L; L = L2; L2 = tmp;
        uint8_t *tm = mark; mark = mark2; mark2 = tm;
        last_changes = changes;
        if (changes == 0) break;
    }
    free(L); free(L2); free(mark); free(mark2); free(cnt); free(prev); free(cut);
    return t;
}
