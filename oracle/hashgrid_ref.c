/* ORACLE — test infrastructure only.  Never linked into the product path.
 *
 * Plain-C restatement of the multires hash-grid encoding of the NGPMT field (tiny-cuda-nn
 * "Grid/Hash", reference models/ngp_mt.py:70-82, L=16 F=2 log2_T=19 N_min=16), forward gather and
 * backward scatter.  It is the same algorithm as oracle/field_ref.py::hash_encode (the torch
 * statement, which stays the primary one; tests/test_oracle_kat.py checks the two agree) — this
 * file exists because the torch statement's per-level index arithmetic made the oracle CPU
 * trainer ~10 s/step, too slow for the PSNR seed ensembles.
 *
 *   pos   = (float)((double)scale * x + 0.5)      (fma(scale, x, 0.5) as field_ref.py computes it)
 *   pg    = (uint32)(int)floor(pos), frac = pos - floor(pos)
 *   index = dense x + y*res + z*res^2 while the stride stays <= params, else
 *           x*1 ^ y*2654435761 ^ z*805459861 (uint32); then % params; + the level's offset
 *   w     = 1 * w_x * w_y * w_z (corner c: bit d of c selects frac_d, else 1 - frac_d)
 *   enc[n][2l+f] = sum_c w_c * table[index_c][f]      (corners summed in order c = 0..7)
 * Backward: dtable[index_c][f] += w_c * denc[n][2l+f], samples in order n = 0..N-1 (serial:
 * the result does not depend on a thread schedule).
 * PARITY UNPINNED w.r.t. tcnn (not vendored; see field_ref.py).
 */
#include <math.h>
#include <stdint.h>

#define NCN_L 16

typedef struct {
    float scale;
    int64_t res, params, offset;
} level_t;

static void load_levels(const float *scales, const int64_t *res, const int64_t *params, const int64_t *offs,
                        level_t *lv) {
    for (int l = 0; l < NCN_L; ++l) {
        lv[l].scale = scales[l];
        lv[l].res = res[l];
        lv[l].params = params[l];
        lv[l].offset = offs[l];
    }
}

/* the 8 corner indices and weights of point x (3 floats in [0,1]) at level lv */
static void corners(const float *x, const level_t *lv, int64_t *idx, float *w) {
    static const uint32_t primes[3] = {1u, 2654435761u, 805459861u};
    uint32_t pg[3];
    float frac[3];
    for (int d = 0; d < 3; ++d) {
        float pos = (float)((double)lv->scale * (double)x[d] + 0.5);
        float fl = floorf(pos);
        frac[d] = pos - fl;
        pg[d] = (uint32_t)(int64_t)fl;
    }
    for (int c = 0; c < 8; ++c) {
        uint32_t p[3];
        float wc = 1.0f;
        for (int d = 0; d < 3; ++d) {
            int bit = (c >> d) & 1;
            p[d] = pg[d] + (uint32_t)bit;
            wc = wc * (bit ? frac[d] : 1.0f - frac[d]);
        }
        uint64_t stride = 1;
        uint32_t index = 0;
        for (int d = 0; d < 3; ++d) {
            if (stride > (uint64_t)lv->params) break;
            index = index + p[d] * (uint32_t)stride;
            stride *= (uint64_t)lv->res;
        }
        if ((uint64_t)lv->params < stride) {
            index = 0;
            for (int d = 0; d < 3; ++d) index ^= p[d] * primes[d];
        }
        idx[c] = (int64_t)(index % (uint32_t)lv->params) + lv->offset;
        w[c] = wc;
    }
}

/* enc (N, 32) = hash_encode(x01 (N,3), table (n_entries, 2)) */
void hashgrid_fwd(const float *x01, int64_t n, const float *table, const float *scales, const int64_t *res,
                  const int64_t *params, const int64_t *offs, float *enc) {
    level_t lv[NCN_L];
    load_levels(scales, res, params, offs, lv);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int64_t idx[8];
        float w[8];
        for (int l = 0; l < NCN_L; ++l) {
            corners(x01 + 3 * i, &lv[l], idx, w);
            float a = 0.0f, b = 0.0f;
            for (int c = 0; c < 8; ++c) {
                a += w[c] * table[2 * idx[c]];
                b += w[c] * table[2 * idx[c] + 1];
            }
            enc[32 * i + 2 * l] = a;
            enc[32 * i + 2 * l + 1] = b;
        }
    }
}

/* dtable (n_entries, 2) += d enc / d table ^T denc (N, 32); serial over samples */
void hashgrid_bwd(const float *x01, int64_t n, const float *denc, const float *scales, const int64_t *res,
                  const int64_t *params, const int64_t *offs, float *dtable) {
    level_t lv[NCN_L];
    load_levels(scales, res, params, offs, lv);
    for (int64_t i = 0; i < n; ++i) {
        int64_t idx[8];
        float w[8];
        for (int l = 0; l < NCN_L; ++l) {
            float ga = denc[32 * i + 2 * l], gb = denc[32 * i + 2 * l + 1];
            if (ga == 0.0f && gb == 0.0f) continue;
            corners(x01 + 3 * i, &lv[l], idx, w);
            for (int c = 0; c < 8; ++c) {
                dtable[2 * idx[c]] += w[c] * ga;
                dtable[2 * idx[c] + 1] += w[c] * gb;
            }
        }
    }
}
