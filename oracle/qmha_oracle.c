/*
 * qmha_oracle.c -- CPU restatement of the reference's attention algorithms.
 *
 * TEST INFRASTRUCTURE ONLY (see qmha_oracle.h).  Built with -ffp-contract=off so
 * that every fused multiply-add below is explicit (fmaf) and mirrors where the
 * reference's nvcc build contracts a*b+c (nvcc default --fmad=true), while the
 * g++-built verify path (utils/verify.cu) has no contraction on x86-64.
 */
#include "qmha_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define GROUP 32 /* Br = Bc = 32, include/config.h:10-11 */

/* ------------------------------------------------------------------------- */
/* small thread pool: run fn(i, ctx) for i in [0, n)                          */
/* ------------------------------------------------------------------------- */
typedef void (*work_fn)(long i, void *ctx);
typedef struct {
    work_fn fn;
    void *ctx;
    long n;
    long next;
    pthread_mutex_t mu;
} pool_t;

static void *pool_worker(void *arg) {
    pool_t *p = (pool_t *)arg;
    for (;;) {
        pthread_mutex_lock(&p->mu);
        long i = p->next++;
        pthread_mutex_unlock(&p->mu);
        if (i >= p->n) break;
        p->fn(i, p->ctx);
    }
    return NULL;
}

static void parallel_for(long n, int nthreads, work_fn fn, void *ctx) {
    if (nthreads <= 0) {
        long c = sysconf(_SC_NPROCESSORS_ONLN);
        nthreads = c > 0 ? (int)c : 1;
    }
    if (nthreads > 64) nthreads = 64;
    if (nthreads > n) nthreads = (int)(n > 0 ? n : 1);
    if (nthreads <= 1) {
        for (long i = 0; i < n; ++i) fn(i, ctx);
        return;
    }
    pool_t p;
    p.fn = fn;
    p.ctx = ctx;
    p.n = n;
    p.next = 0;
    pthread_mutex_init(&p.mu, NULL);
    pthread_t th[64];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, pool_worker, &p);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&p.mu);
}

/* ------------------------------------------------------------------------- */
/* utils/verify.cu                                                            */
/* ------------------------------------------------------------------------- */

/* verify.cu:9-23 (apply_rope_cpu), float math: std::pow/sin/cos on float args. */
static void rope_row(float *row, int pos, int d) {
    const float base = 10000.0f;
    for (int k = 0; k < d / 2; ++k) {
        float theta = powf(base, -(float)(2 * k) / d);
        float angle = pos * theta;
        float sin_a = sinf(angle);
        float cos_a = cosf(angle);
        float x = row[k];
        float y = row[k + d / 2];
        row[k] = x * cos_a - y * sin_a;
        row[k + d / 2] = x * sin_a + y * cos_a;
    }
}

/* verify.cu:25-104 (cpu_reference) */
void oracle_cpu_reference_rope(const float *Q, const float *K, const float *V, float *out,
                               int N, int d_model, int h) {
    int dh = d_model / h;
    float alpha = 1.0f / sqrtf((float)dh);
    float *q_row = (float *)malloc(sizeof(float) * dh);
    float *k_row = (float *)malloc(sizeof(float) * dh);
    float *v_row = (float *)malloc(sizeof(float) * dh);
    float *scores = (float *)malloc(sizeof(float) * N);
    float *sm = (float *)malloc(sizeof(float) * N);
    memset(out, 0, sizeof(float) * (size_t)N * d_model);
    for (int head = 0; head < h; ++head) {
        int col_off = head * dh;
        for (int i = 0; i < N; ++i) {
            for (int kk = 0; kk < dh; ++kk) q_row[kk] = Q[(size_t)i * d_model + col_off + kk];
            rope_row(q_row, i, dh);
            float max_score = -INFINITY;
            for (int j = 0; j < N; ++j) {
                for (int kk = 0; kk < dh; ++kk) k_row[kk] = K[(size_t)j * d_model + col_off + kk];
                rope_row(k_row, j, dh);
                float s = 0.0f;
                for (int kk = 0; kk < dh; ++kk) s += q_row[kk] * k_row[kk];
                s *= alpha;
                scores[j] = s;
                if (s > max_score) max_score = s;
            }
            float sum_exp = 0.0f;
            for (int j = 0; j < N; ++j) {
                float e = expf(scores[j] - max_score);
                sm[j] = e;
                sum_exp += e;
            }
            for (int j = 0; j < N; ++j) sm[j] /= sum_exp;
            for (int kk = 0; kk < dh; ++kk) v_row[kk] = 0.0f;
            for (int j = 0; j < N; ++j) {
                float w = sm[j];
                for (int kk = 0; kk < dh; ++kk) v_row[kk] += w * V[(size_t)j * d_model + col_off + kk];
            }
            for (int kk = 0; kk < dh; ++kk) out[(size_t)i * d_model + col_off + kk] = v_row[kk];
        }
    }
    free(q_row);
    free(k_row);
    free(v_row);
    free(scores);
    free(sm);
}

/* verify.cu:153-172 (verify_results) */
long oracle_verify_results(const float *got, const float *ref, size_t n, float eps, float rel) {
    for (size_t i = 0; i < n; ++i) {
        float a = got[i], b = ref[i];
        if (!isfinite(a) || !isfinite(b)) return (long)i;
        float tol = fmaxf(eps, rel * fabsf(b));
        if (fabsf(a - b) > tol) return (long)i;
    }
    return -1;
}

/* ------------------------------------------------------------------------- */
/* tests/generate_golden.cpp:23-92 (softmax_rowwise + cpu_mha)                */
/* ------------------------------------------------------------------------- */
typedef struct {
    const float *Q, *K, *V;
    float *out;
    int B, N, d_model, h;
} attn_ctx;

static void cpu_attention_item(long item, void *vctx) {
    attn_ctx *c = (attn_ctx *)vctx;
    int N = c->N, dm = c->d_model, dh = c->d_model / c->h;
    int b = (int)(item / c->h), head = (int)(item % c->h);
    const float *Q = c->Q + (size_t)b * N * dm + head * dh;
    const float *K = c->K + (size_t)b * N * dm + head * dh;
    const float *V = c->V + (size_t)b * N * dm + head * dh;
    float *O = c->out + (size_t)b * N * dm + head * dh;
    float scale = 1.0f / sqrtf((float)dh);
    float *row = (float *)malloc(sizeof(float) * N);
    for (int i = 0; i < N; ++i) {
        for (int j = 0; j < N; ++j) {
            float s = 0.0f;
            for (int d = 0; d < dh; ++d) s += Q[(size_t)i * dm + d] * K[(size_t)j * dm + d];
            row[j] = s * scale;
        }
        float m = -INFINITY;
        for (int j = 0; j < N; ++j) m = fmaxf(m, row[j]); /* std::max: NaN-free inputs */
        float s = 0.0f;
        for (int j = 0; j < N; ++j) {
            row[j] = expf(row[j] - m);
            s += row[j];
        }
        if (s == 0.0f) s = 1.0f;
        for (int j = 0; j < N; ++j) row[j] /= s;
        for (int d = 0; d < dh; ++d) {
            float acc = 0.0f;
            for (int k = 0; k < N; ++k) acc += row[k] * V[(size_t)k * dm + d];
            O[(size_t)i * dm + d] = acc;
        }
    }
    free(row);
}

void oracle_cpu_attention(const float *Q, const float *K, const float *V, float *out,
                          int B, int N, int d_model, int h, int nthreads) {
    attn_ctx c = {Q, K, V, out, B, N, d_model, h};
    parallel_for((long)B * h, nthreads, cpu_attention_item, &c);
}

/* ------------------------------------------------------------------------- */
/* fp16 helpers (__float2half = round to nearest even)                        */
/* ------------------------------------------------------------------------- */
uint16_t oracle_f32_to_f16(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    uint32_t sign = (u >> 16) & 0x8000u;
    uint32_t exp = (u >> 23) & 0xffu;
    uint32_t man = u & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (man ? 0x200u : 0u));
    int e = (int)exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        int shift = 14 - e; /* 1 - e + 13 */
        uint32_t half_man = man >> shift;
        uint32_t rem = man & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (half_man & 1u))) half_man++;
        return (uint16_t)(sign | half_man);
    }
    uint32_t half_man = man >> 13;
    uint32_t rem = man & 0x1fffu;
    uint32_t r = sign | ((uint32_t)e << 10) | half_man;
    if (rem > 0x1000u || (rem == 0x1000u && (half_man & 1u))) r++; /* may carry into exponent: correct */
    return (uint16_t)r;
}

float oracle_f16_to_f32(uint16_t hb) {
    uint32_t sign = ((uint32_t)hb & 0x8000u) << 16;
    uint32_t exp = (hb >> 10) & 0x1fu;
    uint32_t man = hb & 0x3ffu;
    uint32_t u;
    if (exp == 0) {
        if (man == 0) {
            u = sign;
        } else {
            int e = -1;
            do {
                man <<= 1;
                e++;
            } while (!(man & 0x400u));
            man &= 0x3ffu;
            u = sign | ((uint32_t)(127 - 15 - e) << 23) | (man << 13);
        }
    } else if (exp == 31) {
        u = sign | 0x7f800000u | (man << 13);
    } else {
        u = sign | ((exp - 15 + 127) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

void oracle_fill_ones(float *x, size_t n) {
    for (size_t i = 0; i < n; ++i) x[i] = 1.0f;
}

/* The reference reduces a row's 32 per-lane values with a __shfl_xor butterfly
 * (shift 16,8,4,2,1; e.g. fa_tc_int8_b.cu:324-326, fa.cu:177-182).  Float add is
 * commutative, so every lane ends with the same value; this reproduces it. */
static float xor_tree_sum32(const float *v_in) {
    float v[32], t[32];
    memcpy(v, v_in, sizeof(v));
    for (int shift = 16; shift >= 1; shift >>= 1) {
        for (int i = 0; i < 32; ++i) t[i] = v[i] + v[i ^ shift];
        memcpy(v, t, sizeof(v));
    }
    return v[0];
}

/* ------------------------------------------------------------------------- */
/* INT8: mha_kernels/fa_tc_int8_b.cu                                          */
/* ------------------------------------------------------------------------- */

/* fa_tc_int8_b.cu:33-152 (fp32_to_int8sram), math only. */
float oracle_quantize_block(const float *src, int rows, int cols, int ld, int8_t *dst, int ldd) {
    float mn = INFINITY, mx = -INFINITY;
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            float v = src[(size_t)r * ld + c];
            mn = fminf(mn, v);
            mx = fmaxf(mx, v);
        }
    float sc = fmaxf(fmaxf(fabsf(mx), fabsf(mn)) / 127.0f, 1e-8f); /* :104 */
    float inv = 1.0f / sc;                                          /* :106 */
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) {
            float scaled = src[(size_t)r * ld + c] * inv; /* :137 */
            float rr = rintf(scaled);                     /* __float2int_rn: RNE */
            /* __float2int_rn (PTX cvt.rni.s32.f32) saturates to the int range and converts NaN to 0
               (fmaxf / fminf would turn a NaN into the clamp bound) */
            int q = rr != rr ? 0 : (int)fmaxf(fminf(rr, 2147483520.0f), -2147483648.0f);
            q = q < -128 ? -128 : (q > 127 ? 127 : q); /* :139 */
            dst[(size_t)r * ldd + c] = (int8_t)q;
        }
    return sc;
}

typedef struct {
    const float *X;
    int B, N, d_model, h;
    int8_t *Xi;
    float *scales;
} qh_ctx;

static void quantize_heads_item(long item, void *vctx) {
    qh_ctx *c = (qh_ctx *)vctx;
    int dh = c->d_model / c->h, G = c->N / GROUP;
    long bh = item / G;
    int g = (int)(item % G);
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const float *src = c->X + ((size_t)b * c->N + (size_t)g * GROUP) * c->d_model + head * dh;
    int8_t *dst = c->Xi + ((size_t)bh * c->N + (size_t)g * GROUP) * dh;
    c->scales[bh * G + g] = oracle_quantize_block(src, GROUP, dh, c->d_model, dst, dh);
}

void oracle_quantize_heads(const float *X, int B, int N, int d_model, int h, int8_t *Xi, float *scales) {
    qh_ctx c = {X, B, N, d_model, h, Xi, scales};
    parallel_for((long)B * h * (N / GROUP), 1, quantize_heads_item, &c);
}

void oracle_qk_int32(const int8_t *Qi, const int8_t *Ki, int N, int d, int32_t *S) {
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            int32_t acc = 0;
            for (int k = 0; k < d; ++k) acc += (int32_t)Qi[(size_t)i * d + k] * (int32_t)Ki[(size_t)j * d + k];
            S[(size_t)i * N + j] = acc;
        }
}

typedef struct {
    int B, N, d_model, h;
    const int8_t *Qi, *Ki, *Vi;
    const float *sQ, *sK, *sV;
    float *out;
} int8_ctx;

/* One 32-row query group of one head: fa_tc_int8_b.cu:408-579 (fa_kernel) with
 * online_softmax_and_accum_output (:247-373), without the smem aliasing of
 * :450-461 and with a private P scale per (q-group, kv-group). */
static void fa_int8_item(long item, void *vctx) {
    int8_ctx *c = (int8_ctx *)vctx;
    int N = c->N, dh = c->d_model / c->h, G = N / GROUP;
    long bh = item / G;
    int g = (int)(item % G);
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const float inv_sqrt_d = 1.0f / sqrtf((float)dh); /* fa_tc_int8_b.cu:587 */
    const int8_t *Qg = c->Qi + ((size_t)bh * N + (size_t)g * GROUP) * dh;
    const float sQ = c->sQ[bh * G + g];

    float *O = (float *)calloc((size_t)GROUP * dh, sizeof(float));
    float l[GROUP], m_prev[GROUP];
    for (int r = 0; r < GROUP; ++r) {
        l[r] = 0.0f;
        m_prev[r] = 0.0f; /* :402, m0 = 0 (not -inf) */
    }
    float s[GROUP][GROUP];
    int8_t Pi[GROUP][GROUP];

    for (int t = 0; t < G; ++t) {
        const int8_t *Kt = c->Ki + ((size_t)bh * N + (size_t)t * GROUP) * dh;
        const int8_t *Vt = c->Vi + ((size_t)bh * N + (size_t)t * GROUP) * dh;
        const float sK = c->sK[bh * G + t], sV = c->sV[bh * G + t];
        /* Q@K^T (int32, :514) + dequant (:176-180) + 1/sqrt(d) (:295) */
        for (int r = 0; r < GROUP; ++r)
            for (int j = 0; j < GROUP; ++j) {
                int32_t acc = 0;
                for (int k = 0; k < dh; ++k) acc += (int32_t)Qg[r * dh + k] * (int32_t)Kt[j * dh + k];
                float deq = (float)acc * sQ * sK;
                s[r][j] = deq * inv_sqrt_d;
            }
        /* online softmax per row (:281-346) */
        for (int r = 0; r < GROUP; ++r) {
            float m_new = m_prev[r];
            for (int j = 0; j < GROUP; ++j) m_new = fmaxf(m_new, s[r][j]);
            float lane[GROUP];
            for (int j = 0; j < GROUP; ++j) {
                s[r][j] = expf(s[r][j] - m_new); /* :315 */
                lane[j] = s[r][j];
            }
            float sum_new = xor_tree_sum32(lane);
            float alpha = expf(m_prev[r] - m_new); /* :329 */
            l[r] = fmaf(alpha, l[r], sum_new);     /* :336, contracted */
            for (int d = 0; d < dh; ++d) O[r * dh + d] *= alpha; /* :344 */
            m_prev[r] = m_new;                                   /* :528-536 */
        }
        /* P quantisation over the 32x32 tile (:359) */
        float sP = oracle_quantize_block(&s[0][0], GROUP, GROUP, GROUP, &Pi[0][0], GROUP);
        /* P@V (int32, :366) and accumulation (:369-371) */
        for (int r = 0; r < GROUP; ++r) {
            for (int d = 0; d < dh; ++d) {
                int32_t acc = 0;
                for (int j = 0; j < GROUP; ++j) acc += (int32_t)Pi[r][j] * (int32_t)Vt[j * dh + d];
                O[r * dh + d] = fmaf((float)acc * sP, sV, O[r * dh + d]);
            }
        }
    }
    float *out = c->out + ((size_t)b * N + (size_t)g * GROUP) * c->d_model + head * dh;
    for (int r = 0; r < GROUP; ++r)
        for (int d = 0; d < dh; ++d)
            out[(size_t)r * c->d_model + d] = (l[r] > 1e-20f) ? O[r * dh + d] / l[r] : 0.0f; /* :549-553 */
    free(O);
}

void oracle_fa_int8(const float *Q, const float *K, const float *V, float *out,
                    int B, int N, int d_model, int h, int nthreads) {
    int dh = d_model / h, G = N / GROUP;
    size_t ne = (size_t)B * h * N * dh, ns = (size_t)B * h * G;
    int8_t *Qi = (int8_t *)malloc(ne), *Ki = (int8_t *)malloc(ne), *Vi = (int8_t *)malloc(ne);
    float *sQ = (float *)malloc(ns * 4), *sK = (float *)malloc(ns * 4), *sV = (float *)malloc(ns * 4);
    oracle_quantize_heads(Q, B, N, d_model, h, Qi, sQ);
    oracle_quantize_heads(K, B, N, d_model, h, Ki, sK);
    oracle_quantize_heads(V, B, N, d_model, h, Vi, sV);
    int8_ctx c = {B, N, d_model, h, Qi, Ki, Vi, sQ, sK, sV, out};
    parallel_for((long)ns, nthreads, fa_int8_item, &c);
    free(Qi);
    free(Ki);
    free(Vi);
    free(sQ);
    free(sK);
    free(sV);
}

/* ------------------------------------------------------------------------- */
/* INT8, per-tensor mode (fa_tc_int8_pt).  NOT a reference kernel: BASELINE.json's
 * "per-tensor Q/K/V quant" wording, offered beside the reference's per-block contract
 * ("a per-tensor mode may be offered as an extra flag").  Same quantiser
 * (fa_tc_int8_b.cu:33-152) applied to each head's whole [N, d] slice -- the matrix the
 * reference's launch<> extracts per head (include/launchers.h:42-52) -- and P quantised with
 * the static scale 1/127, so the P@V products of every tile share one unit and O accumulates as
 * the int32 sums, rescaled by alpha only.  The contract is stated in base 2 with the score
 * constant the kernel uses (r06; this mode has no reference numerics to follow):
 *   c = RN22(sQ * RN(RN(1/sqrt(d)) * log2 e) * sK)   (float products; RN22: 22 significant bits)
 *   x = RN(S * c - m)   (S the int32 Q.K, one rounding: the kernel's fused multiply-add),
 *   row max xm = RN(S_max * c); lazy base m: max(0, xm) on tile 0 (m0 = 0, the exact rule); on a later
 *   tile it moves to xm only when the p of one of the row's key parts (the kernel's lanes, summed in its
 *   order: quarters of eight keys at d = 64, halves of sixteen elsewhere) sum above 2047/127 -- then the tile's p are
 *   recomputed -- so p <= 2047/127,  Pi = min(rint(127 p), 2047),  alpha = 2^(m_old - m_new),
 *   l = alpha l + sum(p) (per key half, joined at the end),  O = alpha O + (float)(Pi.Vi)[int32],
 *   out = l > 1e-20 ? (O * (sV / 127)) / l : 0.                                   */
/* ------------------------------------------------------------------------- */
typedef struct {
    const float *X;
    int B, N, d_model, h;
    int8_t *Xi;
    float *scales;
} qt_ctx;

static void quantize_tensor_item(long bh, void *vctx) {
    qt_ctx *c = (qt_ctx *)vctx;
    int dh = c->d_model / c->h;
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const float *src = c->X + (size_t)b * c->N * c->d_model + head * dh;
    c->scales[bh] = oracle_quantize_block(src, c->N, dh, c->d_model, c->Xi + (size_t)bh * c->N * dh, dh);
}

void oracle_quantize_heads_pt(const float *X, int B, int N, int d_model, int h, int8_t *Xi, float *scales) {
    qt_ctx c = {X, B, N, d_model, h, Xi, scales};
    parallel_for((long)B * h, 0, quantize_tensor_item, &c);
}

static float tree_sum16_of(const float *p) { /* the kernel's tree_sum16 order */
    float a = (p[0] + p[1]) + (p[2] + p[3]), b = (p[4] + p[5]) + (p[6] + p[7]);
    float c = (p[8] + p[9]) + (p[10] + p[11]), d = (p[12] + p[13]) + (p[14] + p[15]);
    return (a + b) + (c + d);
}
#define PT_SUM_CAP (2047.0f / 127.0f) /* the kernel's kPtSumCap */
/* the kernel's score constant (qmha_fa_int8.hip: c_log2 on the host, cq, c_pt) */
static float pt_score_constant(float sQ, float sK, int dh) {
    const float c_log2 = (1.0f / sqrtf((float)dh)) * 1.4426950408889634f;
    const float cq = sQ * c_log2;
    const float c = cq * sK;
    uint32_t u;
    memcpy(&u, &c, 4);
    u = (u + 2u) & ~3u; /* 22 significant bits, ties away from zero (c >= 0) */
    float r;
    memcpy(&r, &u, 4);
    return r;
}
static void fa_int8_pt_item(long item, void *vctx) {
    int8_ctx *c = (int8_ctx *)vctx;
    int N = c->N, dh = c->d_model / c->h, G = N / GROUP;
    long bh = item / G;
    int g = (int)(item % G);
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const int8_t *Qg = c->Qi + ((size_t)bh * N + (size_t)g * GROUP) * dh;
    const float sV = c->sV[bh];
    const float cc = pt_score_constant(c->sQ[bh], c->sK[bh], dh);

    float *O = (float *)calloc((size_t)GROUP * dh, sizeof(float));
    const int quarters = dh == 64; /* the 16x16 kernel's lane parts (d = 64); halves elsewhere */
    const int nparts = quarters ? 4 : 2;
    float l[GROUP][4], m_prev[GROUP];
    for (int r = 0; r < GROUP; ++r) {
        l[r][0] = l[r][1] = l[r][2] = l[r][3] = 0.0f;
        m_prev[r] = 0.0f; /* m0 = 0, as fa_tc_int8_b.cu:402 */
    }
    int32_t S[GROUP][GROUP];
    for (int t = 0; t < G; ++t) {
        const int8_t *Kt = c->Ki + ((size_t)bh * N + (size_t)t * GROUP) * dh;
        const int8_t *Vt = c->Vi + ((size_t)bh * N + (size_t)t * GROUP) * dh;
        for (int r = 0; r < GROUP; ++r)
            for (int j = 0; j < GROUP; ++j) {
                int32_t acc = 0;
                for (int k = 0; k < dh; ++k) acc += (int32_t)Qg[r * dh + k] * (int32_t)Kt[j * dh + k];
                S[r][j] = acc;
            }
        for (int r = 0; r < GROUP; ++r) {
            /* lazy base (r06): tile 0 takes max(m0, row max); later tiles move the base to the row max only
             * when one of the row's key parts (the kernel's lanes: quarters at d = 64, halves elsewhere) sums
             * above the cap, so p <= 2047/127 and Pi <= 2047 */
            int32_t smax = S[r][0];
            for (int j = 1; j < GROUP; ++j) smax = S[r][j] > smax ? S[r][j] : smax;
            const float xm = (float)smax * cc;
            float alpha = 1.0f;
            if (t == 0) m_prev[r] = fmaxf(m_prev[r], xm);
            float p[GROUP], ts[4];
            for (int pass = 0; pass < 2; ++pass) {
                for (int j = 0; j < GROUP; ++j) /* S * cc is exact in double (< 53 bits): one rounding */
                    p[j] = exp2f((float)((double)S[r][j] * (double)cc - (double)m_prev[r]));
                int over = 0;
                for (int hh = 0; hh < nparts; ++hh) {
                    if (quarters) { /* lane group hh: keys kap16(j >> 2, 4 hh + (j & 3)), summed as a tree */
                        float q[8];
                        for (int j = 0; j < 8; ++j) {
                            const int mm = 4 * hh + (j & 3);
                            q[j] = p[16 * (mm >> 3) + 4 * ((mm >> 2) & 1) + (mm & 3) + 8 * (j >> 2)];
                        }
                        ts[hh] = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
                    } else { /* lane half hh: keys (i & 3) + 8 (i >> 2) + 4 hh */
                        float p16[16];
                        for (int i = 0; i < 16; ++i) p16[i] = p[(i & 3) + 8 * (i >> 2) + 4 * hh];
                        ts[hh] = tree_sum16_of(p16);
                    }
                    over |= ts[hh] > PT_SUM_CAP;
                }
                if (pass == 1 || t == 0 || !over) break;
                alpha = exp2f(m_prev[r] - xm);
                m_prev[r] = xm;
            }
            for (int hh = 0; hh < nparts; ++hh) l[r][hh] = fmaf(alpha, l[r][hh], ts[hh]);
            for (int d = 0; d < dh; ++d) O[r * dh + d] *= alpha;
            int Pi[GROUP];
            for (int j = 0; j < GROUP; ++j) {
                float rr = rintf(p[j] * 127.0f); /* static P scale 1/127; p in [0, 16] */
                Pi[j] = rr != rr ? 0 : (int)fminf(rr, 2047.0f);
            }
            for (int d = 0; d < dh; ++d) {
                int32_t acc = 0;
                for (int j = 0; j < GROUP; ++j) acc += Pi[j] * (int32_t)Vt[j * dh + d];
                O[r * dh + d] += (float)acc;
            }
        }
    }
    const float sVq = sV / 127.0f;
    float *out = c->out + ((size_t)b * N + (size_t)g * GROUP) * c->d_model + head * dh;
    for (int r = 0; r < GROUP; ++r)
        for (int d = 0; d < dh; ++d)
        {
            const float lr = quarters ? (l[r][0] + l[r][1]) + (l[r][2] + l[r][3]) : l[r][0] + l[r][1];
            out[(size_t)r * c->d_model + d] = (lr > 1e-20f) ? (O[r * dh + d] * sVq) / lr : 0.0f;
        }
    free(O);
}

void oracle_fa_int8_pt(const float *Q, const float *K, const float *V, float *out,
                       int B, int N, int d_model, int h, int nthreads) {
    int dh = d_model / h;
    size_t ne = (size_t)B * h * N * dh, nbh = (size_t)B * h;
    int8_t *Qi = (int8_t *)malloc(ne), *Ki = (int8_t *)malloc(ne), *Vi = (int8_t *)malloc(ne);
    float *sQ = (float *)malloc(nbh * 4), *sK = (float *)malloc(nbh * 4), *sV = (float *)malloc(nbh * 4);
    oracle_quantize_heads_pt(Q, B, N, d_model, h, Qi, sQ);
    oracle_quantize_heads_pt(K, B, N, d_model, h, Ki, sK);
    oracle_quantize_heads_pt(V, B, N, d_model, h, Vi, sV);
    int8_ctx c = {B, N, d_model, h, Qi, Ki, Vi, sQ, sK, sV, out};
    parallel_for((long)nbh * (N / GROUP), nthreads, fa_int8_pt_item, &c);
    free(Qi);
    free(Ki);
    free(Vi);
    free(sQ);
    free(sK);
    free(sV);
}

/* ------------------------------------------------------------------------- */
/* FP16: mha_kernels/fa_tc_v1a.cu                                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    const float *Q, *K, *V;
    float *out;
    int B, N, d_model, h;
} fa_ctx;

static void fa_fp16_item(long item, void *vctx) {
    fa_ctx *c = (fa_ctx *)vctx;
    int N = c->N, dm = c->d_model, dh = dm / c->h, G = N / GROUP;
    long bh = item / G;
    int g = (int)(item % G);
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const float inv_sqrt_d = 1.0f / sqrtf((float)dh); /* fa_tc_v1a.cu:421 */
    const float *Qb = c->Q + (size_t)b * N * dm + head * dh;
    const float *Kb = c->K + (size_t)b * N * dm + head * dh;
    const float *Vb = c->V + (size_t)b * N * dm + head * dh;

    float *q = (float *)malloc(sizeof(float) * GROUP * dh); /* half(Q) as float, :267 */
    float *kt = (float *)malloc(sizeof(float) * GROUP * dh);
    float *vv = (float *)malloc(sizeof(float) * GROUP * dh);
    float *O = (float *)calloc((size_t)GROUP * dh, sizeof(float));
    float l[GROUP], m_prev[GROUP], s[GROUP][GROUP], ph[GROUP][GROUP];
    for (int r = 0; r < GROUP; ++r) {
        l[r] = 0.0f;
        m_prev[r] = 0.0f; /* :290 */
        for (int d = 0; d < dh; ++d)
            q[r * dh + d] = oracle_f16_to_f32(oracle_f32_to_f16(Qb[(size_t)(g * GROUP + r) * dm + d]));
    }
    for (int t = 0; t < G; ++t) {
        for (int j = 0; j < GROUP; ++j)
            for (int d = 0; d < dh; ++d) {
                kt[j * dh + d] = oracle_f16_to_f32(oracle_f32_to_f16(Kb[(size_t)(t * GROUP + j) * dm + d])); /* :321 */
                vv[j * dh + d] = oracle_f16_to_f32(oracle_f32_to_f16(Vb[(size_t)(t * GROUP + j) * dm + d])); /* :348 */
            }
        /* WMMA f16 x f16 -> f32 (:332): products are exact in fp32; summed in k order. */
        for (int r = 0; r < GROUP; ++r)
            for (int j = 0; j < GROUP; ++j) {
                float acc = 0.0f;
                for (int d = 0; d < dh; ++d) acc = fmaf(q[r * dh + d], kt[j * dh + d], acc);
                s[r][j] = acc * inv_sqrt_d; /* :140 */
            }
        for (int r = 0; r < GROUP; ++r) {
            float m_new = m_prev[r];
            for (int j = 0; j < GROUP; ++j) m_new = fmaxf(m_new, s[r][j]);
            float lane[GROUP];
            for (int j = 0; j < GROUP; ++j) {
                float p = expf(s[r][j] - m_new);                        /* :169 */
                lane[j] = p;                                            /* sum uses fp32 p, :171 */
                ph[r][j] = oracle_f16_to_f32(oracle_f32_to_f16(p));     /* :174 */
            }
            float sum_new = xor_tree_sum32(lane);
            float alpha = expf(m_prev[r] - m_new); /* :195 */
            l[r] = fmaf(alpha, l[r], sum_new);     /* :198, contracted */
            for (int d = 0; d < dh; ++d) O[r * dh + d] *= alpha; /* :207 */
            m_prev[r] = m_new;
        }
        /* O += P_f16 @ V_f16 via WMMA add_to_output (:78-87, :218): c = PV; c += O */
        for (int r = 0; r < GROUP; ++r)
            for (int d = 0; d < dh; ++d) {
                float acc = 0.0f;
                for (int j = 0; j < GROUP; ++j) acc = fmaf(ph[r][j], vv[j * dh + d], acc);
                O[r * dh + d] = acc + O[r * dh + d];
            }
    }
    float *out = c->out + ((size_t)b * N + (size_t)g * GROUP) * dm + head * dh;
    for (int r = 0; r < GROUP; ++r)
        for (int d = 0; d < dh; ++d)
            out[(size_t)r * dm + d] = (l[r] > 1e-10f) ? O[r * dh + d] / l[r] : 0.0f; /* :384-388 */
    free(q);
    free(kt);
    free(vv);
    free(O);
}

void oracle_fa_fp16(const float *Q, const float *K, const float *V, float *out,
                    int B, int N, int d_model, int h, int nthreads) {
    fa_ctx c = {Q, K, V, out, B, N, d_model, h};
    parallel_for((long)B * h * (N / GROUP), nthreads, fa_fp16_item, &c);
}

/* The fp16 GPU kernel's own contract (r06): fa_tc_v1a's arithmetic with the softmax in
 * base 2 (x = S * (1/sqrtf(d)) * log2 e, exp2) and a LAZY base: p = exp2(x - m) against a per-row base m
 * (m0 = 0) that moves to the tile's row max only when the p of one of the row's key parts sum above 2^12
 * on that tile; then O and l are scaled by exp2(m_old - m_new) and the tile's p recomputed.  The parts
 * are the kernel's lanes: at d = 64 / 128 (the 16x16x32 kernel) four quarters of eight keys, lane group g
 * holding keys kap16(j >> 2, 4 g + (j & 3)); at other d (the 32x32x16 kernel) two halves of sixteen, keys
 * j with bit 2 of j clear / set.  l is kept per part and summed in the kernel's order.  The reference (oracle_fa_fp16 above) moves m
 * on every tile; the two differ only in the rounding of half(p).  Used by the tests to pin the kernel
 * tightly (the reference bound is checked against oracle_fa_fp16). */
static void fa_fp16_lazy_item(long item, void *vctx) {
    fa_ctx *c = (fa_ctx *)vctx;
    int N = c->N, dm = c->d_model, dh = dm / c->h, G = N / GROUP;
    long bh = item / G;
    int g = (int)(item % G);
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const float c_log2 = (1.0f / sqrtf((float)dh)) * 1.4426950408889634f; /* the kernel's score constant */
    const float cap = 4096.0f; /* the kernel's kLazySumCap */
    const float *Qb = c->Q + (size_t)b * N * dm + head * dh;
    const float *Kb = c->K + (size_t)b * N * dm + head * dh;
    const float *Vb = c->V + (size_t)b * N * dm + head * dh;
    float *q = (float *)malloc(sizeof(float) * GROUP * dh);
    float *kt = (float *)malloc(sizeof(float) * GROUP * dh);
    float *vv = (float *)malloc(sizeof(float) * GROUP * dh);
    float *O = (float *)calloc((size_t)GROUP * dh, sizeof(float));
    const int quarters = dh == 64 || dh == 128; /* the 16x16x32 kernel's lane parts */
    const int nparts = quarters ? 4 : 2;
    float l[GROUP][4], m[GROUP], s[GROUP][GROUP], ph[GROUP][GROUP];
    for (int r = 0; r < GROUP; ++r) {
        l[r][0] = l[r][1] = l[r][2] = l[r][3] = 0.0f;
        m[r] = 0.0f;
        for (int d = 0; d < dh; ++d)
            q[r * dh + d] = oracle_f16_to_f32(oracle_f32_to_f16(Qb[(size_t)(g * GROUP + r) * dm + d]));
    }
    for (int t = 0; t < G; ++t) {
        for (int j = 0; j < GROUP; ++j)
            for (int d = 0; d < dh; ++d) {
                kt[j * dh + d] = oracle_f16_to_f32(oracle_f32_to_f16(Kb[(size_t)(t * GROUP + j) * dm + d]));
                vv[j * dh + d] = oracle_f16_to_f32(oracle_f32_to_f16(Vb[(size_t)(t * GROUP + j) * dm + d]));
            }
        for (int r = 0; r < GROUP; ++r)
            for (int j = 0; j < GROUP; ++j) {
                float acc = 0.0f;
                for (int d = 0; d < dh; ++d) acc = fmaf(q[r * dh + d], kt[j * dh + d], acc);
                s[r][j] = acc; /* raw S: the kernel scales inside the exponent */
            }
        for (int r = 0; r < GROUP; ++r) {
            float p[GROUP], ts[4];
            for (int pass = 0; pass < 2; ++pass) {
                for (int j = 0; j < GROUP; ++j) p[j] = exp2f(fmaf(s[r][j], c_log2, -m[r]));
                int over = 0;
                for (int hh = 0; hh < nparts; ++hh) {
                    if (quarters) { /* lane group hh: keys kap16(j >> 2, 4 hh + (j & 3)), summed as a tree */
                        float q[8];
                        for (int j = 0; j < 8; ++j) {
                            const int mm = 4 * hh + (j & 3);
                            q[j] = p[16 * (mm >> 3) + 4 * ((mm >> 2) & 1) + (mm & 3) + 8 * (j >> 2)];
                        }
                        ts[hh] = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
                    } else { /* lane half hh: keys (i & 3) + 8 (i >> 2) + 4 hh */
                        float ph16[16];
                        for (int i = 0; i < 16; ++i) ph16[i] = p[(i & 3) + 8 * (i >> 2) + 4 * hh];
                        ts[hh] = tree_sum16_of(ph16);
                    }
                    over |= ts[hh] > cap;
                }
                if (pass == 1 || !over) break;
                float mx = s[r][0]; /* rebase: the row max, O and l scaled, the tile recomputed */
                for (int j = 1; j < GROUP; ++j) mx = fmaxf(mx, s[r][j]);
                const float xm = mx * c_log2;
                const float alpha = exp2f(m[r] - xm);
                for (int hh = 0; hh < nparts; ++hh) l[r][hh] *= alpha;
                for (int d = 0; d < dh; ++d) O[r * dh + d] *= alpha;
                m[r] = xm;
            }
            for (int j = 0; j < GROUP; ++j) ph[r][j] = oracle_f16_to_f32(oracle_f32_to_f16(p[j]));
            for (int hh = 0; hh < nparts; ++hh) l[r][hh] += ts[hh];
        }
        for (int r = 0; r < GROUP; ++r)
            for (int d = 0; d < dh; ++d) {
                float acc = 0.0f;
                for (int j = 0; j < GROUP; ++j) acc = fmaf(ph[r][j], vv[j * dh + d], acc);
                O[r * dh + d] = acc + O[r * dh + d];
            }
    }
    float *out = c->out + ((size_t)b * N + (size_t)g * GROUP) * dm + head * dh;
    for (int r = 0; r < GROUP; ++r)
        for (int d = 0; d < dh; ++d) {
            const float lr = quarters ? (l[r][0] + l[r][1]) + (l[r][2] + l[r][3]) : l[r][0] + l[r][1];
            out[(size_t)r * dm + d] = (lr > 1e-10f) ? O[r * dh + d] / lr : 0.0f;
        }
    free(q);
    free(kt);
    free(vv);
    free(O);
}

void oracle_fa_fp16_lazy(const float *Q, const float *K, const float *V, float *out,
                         int B, int N, int d_model, int h, int nthreads) {
    fa_ctx c = {Q, K, V, out, B, N, d_model, h};
    parallel_for((long)B * h * (N / GROUP), nthreads, fa_fp16_lazy_item, &c);
}

/* ------------------------------------------------------------------------- */
/* FP32 scalar: mha_kernels/fa.cu                                             */
/* ------------------------------------------------------------------------- */
static void fa_fp32_item(long item, void *vctx) {
    fa_ctx *c = (fa_ctx *)vctx;
    int N = c->N, dm = c->d_model, dh = dm / c->h, G = N / GROUP;
    long bh = item / G;
    int g = (int)(item % G);
    int b = (int)(bh / c->h), head = (int)(bh % c->h);
    const float inv_sqrt_d = 1.0f / sqrtf((float)dh); /* fa.cu:410 */
    const float *Qb = c->Q + (size_t)b * N * dm + head * dh;
    const float *Kb = c->K + (size_t)b * N * dm + head * dh;
    const float *Vb = c->V + (size_t)b * N * dm + head * dh;
    float *O = (float *)calloc((size_t)GROUP * dh, sizeof(float));
    float l[GROUP], m_prev[GROUP], s[GROUP][GROUP];
    for (int r = 0; r < GROUP; ++r) {
        l[r] = 0.0f;
        m_prev[r] = 0.0f; /* :279 */
    }
    for (int t = 0; t < G; ++t) {
        /* matmul_warp_tiled (:24-102): acc += a*b over k in order, contracted to fma */
        for (int r = 0; r < GROUP; ++r)
            for (int j = 0; j < GROUP; ++j) {
                float acc = 0.0f;
                const float *qr = Qb + (size_t)(g * GROUP + r) * dm;
                const float *kr = Kb + (size_t)(t * GROUP + j) * dm;
                for (int d = 0; d < dh; ++d) acc = fmaf(qr[d], kr[d], acc);
                s[r][j] = acc * inv_sqrt_d; /* :141 */
            }
        for (int r = 0; r < GROUP; ++r) {
            float m_new = m_prev[r];
            for (int j = 0; j < GROUP; ++j) m_new = fmaxf(m_new, s[r][j]);
            float lane[GROUP];
            for (int j = 0; j < GROUP; ++j) {
                s[r][j] = expf(s[r][j] - m_new); /* :167 */
                lane[j] = s[r][j];
            }
            float sum_new = xor_tree_sum32(lane);
            float alpha = expf(m_prev[r] - m_new); /* :187 */
            l[r] = fmaf(alpha, l[r], sum_new);     /* :190, contracted */
            for (int d = 0; d < dh; ++d) O[r * dh + d] *= alpha; /* :199 */
            m_prev[r] = m_new;
        }
        /* O += P @ V: acc = fma chain over the 32 kv of the tile, then C += acc (:93-94) */
        for (int r = 0; r < GROUP; ++r)
            for (int d = 0; d < dh; ++d) {
                float acc = 0.0f;
                for (int j = 0; j < GROUP; ++j) acc = fmaf(s[r][j], Vb[(size_t)(t * GROUP + j) * dm + d], acc);
                O[r * dh + d] += acc;
            }
    }
    float *out = c->out + ((size_t)b * N + (size_t)g * GROUP) * dm + head * dh;
    for (int r = 0; r < GROUP; ++r)
        for (int d = 0; d < dh; ++d)
            out[(size_t)r * dm + d] = (l[r] > 1e-10f) ? O[r * dh + d] / l[r] : 0.0f; /* :371-375 */
    free(O);
}

void oracle_fa_fp32(const float *Q, const float *K, const float *V, float *out,
                    int B, int N, int d_model, int h, int nthreads) {
    fa_ctx c = {Q, K, V, out, B, N, d_model, h};
    parallel_for((long)B * h * (N / GROUP), nthreads, fa_fp32_item, &c);
}
