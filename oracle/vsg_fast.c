/*
 * vsg_fast.c — host-ISA metric kernels for the CPU-baseline leg (TEST
 * INFRASTRUCTURE ONLY; loaded with the oracle, never by the product).
 *
 * usearch reaches its metrics through SimSIMD, which dispatches at run time to
 * the widest ISA the host has (AVX-512 + FMA on the Zen 5 hosts of the GPU
 * boxes).  This translation unit does the same so that the timed CPU baseline
 * is a fair stand-in for usearch: AVX-512F with fused
 * multiply-add and four independent accumulators, AVX2 + FMA otherwise, a
 * plain loop as the last resort.  Results differ from the parity metrics of
 * vsg_oracle.c (serial, no FMA) in the last bits; the parity tests use those.
 */
#include <immintrin.h>
#include <math.h>
#include <stddef.h>

#define ORC_L2SQ 0
#define ORC_IP 1

static float finish(int metric, float s, float na, float nb) {
    if (metric == ORC_L2SQ) return s;
    if (metric == ORC_IP) return 1.f - s;
    if (na == 0.f && nb == 0.f) return 0.f;
    if (na == 0.f || nb == 0.f) return 1.f;
    return 1.f - s / (sqrtf(na) * sqrtf(nb));
}

__attribute__((target("avx512f,fma"))) static float dist_avx512(int metric, const float* a, const float* b,
                                                                size_t dim) {
    __m512 s0 = _mm512_setzero_ps(), s1 = _mm512_setzero_ps(), s2 = _mm512_setzero_ps(), s3 = _mm512_setzero_ps();
    __m512 na0 = _mm512_setzero_ps(), na1 = _mm512_setzero_ps(), nb0 = _mm512_setzero_ps(), nb1 = _mm512_setzero_ps();
    size_t i = 0;
    if (metric == ORC_L2SQ) {
        for (; i + 64 <= dim; i += 64) {
            __m512 d0 = _mm512_sub_ps(_mm512_loadu_ps(a + i), _mm512_loadu_ps(b + i));
            __m512 d1 = _mm512_sub_ps(_mm512_loadu_ps(a + i + 16), _mm512_loadu_ps(b + i + 16));
            __m512 d2 = _mm512_sub_ps(_mm512_loadu_ps(a + i + 32), _mm512_loadu_ps(b + i + 32));
            __m512 d3 = _mm512_sub_ps(_mm512_loadu_ps(a + i + 48), _mm512_loadu_ps(b + i + 48));
            s0 = _mm512_fmadd_ps(d0, d0, s0);
            s1 = _mm512_fmadd_ps(d1, d1, s1);
            s2 = _mm512_fmadd_ps(d2, d2, s2);
            s3 = _mm512_fmadd_ps(d3, d3, s3);
        }
        for (; i + 16 <= dim; i += 16) {
            __m512 d = _mm512_sub_ps(_mm512_loadu_ps(a + i), _mm512_loadu_ps(b + i));
            s0 = _mm512_fmadd_ps(d, d, s0);
        }
        if (i < dim) {
            const __mmask16 m = (__mmask16)((1u << (dim - i)) - 1u);
            __m512 d = _mm512_sub_ps(_mm512_maskz_loadu_ps(m, a + i), _mm512_maskz_loadu_ps(m, b + i));
            s0 = _mm512_fmadd_ps(d, d, s0);
        }
    } else if (metric == ORC_IP) {
        for (; i + 64 <= dim; i += 64) {
            s0 = _mm512_fmadd_ps(_mm512_loadu_ps(a + i), _mm512_loadu_ps(b + i), s0);
            s1 = _mm512_fmadd_ps(_mm512_loadu_ps(a + i + 16), _mm512_loadu_ps(b + i + 16), s1);
            s2 = _mm512_fmadd_ps(_mm512_loadu_ps(a + i + 32), _mm512_loadu_ps(b + i + 32), s2);
            s3 = _mm512_fmadd_ps(_mm512_loadu_ps(a + i + 48), _mm512_loadu_ps(b + i + 48), s3);
        }
        for (; i + 16 <= dim; i += 16) s0 = _mm512_fmadd_ps(_mm512_loadu_ps(a + i), _mm512_loadu_ps(b + i), s0);
        if (i < dim) {
            const __mmask16 m = (__mmask16)((1u << (dim - i)) - 1u);
            s0 = _mm512_fmadd_ps(_mm512_maskz_loadu_ps(m, a + i), _mm512_maskz_loadu_ps(m, b + i), s0);
        }
    } else {
        for (; i + 32 <= dim; i += 32) {
            __m512 a0 = _mm512_loadu_ps(a + i), a1 = _mm512_loadu_ps(a + i + 16);
            __m512 b0 = _mm512_loadu_ps(b + i), b1 = _mm512_loadu_ps(b + i + 16);
            s0 = _mm512_fmadd_ps(a0, b0, s0);
            s1 = _mm512_fmadd_ps(a1, b1, s1);
            na0 = _mm512_fmadd_ps(a0, a0, na0);
            na1 = _mm512_fmadd_ps(a1, a1, na1);
            nb0 = _mm512_fmadd_ps(b0, b0, nb0);
            nb1 = _mm512_fmadd_ps(b1, b1, nb1);
        }
        for (; i < dim; i += 16) {
            const size_t r = dim - i;
            const __mmask16 m = r >= 16 ? (__mmask16)0xFFFF : (__mmask16)((1u << r) - 1u);
            __m512 a0 = _mm512_maskz_loadu_ps(m, a + i), b0 = _mm512_maskz_loadu_ps(m, b + i);
            s0 = _mm512_fmadd_ps(a0, b0, s0);
            na0 = _mm512_fmadd_ps(a0, a0, na0);
            nb0 = _mm512_fmadd_ps(b0, b0, nb0);
        }
    }
    const float s = _mm512_reduce_add_ps(_mm512_add_ps(_mm512_add_ps(s0, s1), _mm512_add_ps(s2, s3)));
    const float na = _mm512_reduce_add_ps(_mm512_add_ps(na0, na1));
    const float nb = _mm512_reduce_add_ps(_mm512_add_ps(nb0, nb1));
    return finish(metric, s, na, nb);
}

__attribute__((target("avx2,fma"))) static float hsum256(__m256 v) {
    __m128 x = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
    x = _mm_add_ps(x, _mm_movehl_ps(x, x));
    x = _mm_add_ss(x, _mm_shuffle_ps(x, x, 1));
    return _mm_cvtss_f32(x);
}

__attribute__((target("avx2,fma"))) static float dist_avx2(int metric, const float* a, const float* b, size_t dim) {
    __m256 s0 = _mm256_setzero_ps(), s1 = _mm256_setzero_ps(), na = _mm256_setzero_ps(), nb = _mm256_setzero_ps();
    size_t i = 0;
    for (; i + 16 <= dim; i += 16) {
        __m256 a0 = _mm256_loadu_ps(a + i), a1 = _mm256_loadu_ps(a + i + 8);
        __m256 b0 = _mm256_loadu_ps(b + i), b1 = _mm256_loadu_ps(b + i + 8);
        if (metric == ORC_L2SQ) {
            __m256 d0 = _mm256_sub_ps(a0, b0), d1 = _mm256_sub_ps(a1, b1);
            s0 = _mm256_fmadd_ps(d0, d0, s0);
            s1 = _mm256_fmadd_ps(d1, d1, s1);
        } else {
            s0 = _mm256_fmadd_ps(a0, b0, s0);
            s1 = _mm256_fmadd_ps(a1, b1, s1);
            if (metric != ORC_IP) {
                na = _mm256_fmadd_ps(a0, a0, _mm256_fmadd_ps(a1, a1, na));
                nb = _mm256_fmadd_ps(b0, b0, _mm256_fmadd_ps(b1, b1, nb));
            }
        }
    }
    float s = hsum256(_mm256_add_ps(s0, s1)), fa = hsum256(na), fb = hsum256(nb);
    for (; i < dim; ++i) {
        if (metric == ORC_L2SQ) {
            const float d = a[i] - b[i];
            s += d * d;
        } else {
            s += a[i] * b[i];
            fa += a[i] * a[i];
            fb += b[i] * b[i];
        }
    }
    return finish(metric, s, fa, fb);
}

static float dist_plain(int metric, const float* a, const float* b, size_t dim) {
    float s = 0.f, na = 0.f, nb = 0.f;
    for (size_t i = 0; i < dim; ++i) {
        if (metric == ORC_L2SQ) {
            const float d = a[i] - b[i];
            s += d * d;
        } else {
            s += a[i] * b[i];
            na += a[i] * a[i];
            nb += b[i] * b[i];
        }
    }
    return finish(metric, s, na, nb);
}

typedef float (*dist_fn)(int, const float*, const float*, size_t);

static dist_fn pick(void) {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f")) return dist_avx512;
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return dist_avx2;
    return dist_plain;
}

static dist_fn g_fn;

float orc_fast_distance(int metric, const float* a, const float* b, size_t dim) {
    dist_fn f = __atomic_load_n(&g_fn, __ATOMIC_RELAXED);
    if (!f) {
        f = pick();
        __atomic_store_n(&g_fn, f, __ATOMIC_RELAXED);
    }
    return f(metric, a, b, dim);
}

const char* orc_fast_isa(void) {
    const dist_fn f = pick();
    return f == dist_avx512 ? "avx512f+fma" : f == dist_avx2 ? "avx2+fma" : "scalar";
}
