// gnnd_sample.hip — on-device synthesis of decoder inputs, in the
// reference's batch layout (graph-major, N = V + C rows per codeword).  Paths relative to
// /root/reference/GNN-decode/.
//
//  * toric / any quantum CSS graph — quantum/error_generate.py:252-278 `gen_syn`: per
//    codeword p is drawn uniformly from a grid, every qubit column flips with probability p
//    (the script's X and Z halves are the same i.i.d. draw), x = [prior log((1-p)/p) at the
//    variable rows, syndrome (-1)^(H^T e) at the check rows], y = e.
//  * AWGN — classical/CGNNI.py:125-147 `Gen_Data` + :157-161 `CustomDataset`: codeword c
//    (a constant word, or a uniform random codeword m G of the code), BPSK 1 - 2c,
//    y' = 1 - 2c + sigma n with sigma^2 = 10^(-SNR/10), x = [LLR 2 y' / sigma^2 at the
//    variable rows, 0 at the check rows], labels c.  SNR cycles over a grid by GLOBAL codeword
//    index.
//
// Randomness: Philox4x32-10 (Salmon et al., SC'11), counter = {word, codeword lo, codeword
// hi, stream}, key = seed.  Counter-based, so a draw depends only on (seed, global codeword
// index): a data-parallel shard [start, end) passes offset = start and the union of the
// shards is bit-identical to one single-GPU draw of the global batch.  The reference draws
// with numpy / torch CPU generators; parity is distributional (tests/test_sample_gpu.py).
//
// Work: HBM-write bound (each codeword writes N + V values, reads nothing but a few KB of
// graph / generator tables that stay in L2).  A workgroup owns a tile of codewords; Bernoulli
// and Gaussian draws come four per Philox call; syndromes use the check CSR on the tile's
// error bits in LDS; random codewords are parities of (message & generator column) words.
#include "gnnd_common.h"

namespace {

constexpr uint32_t kPhiloxM0 = 0xD2511F53u, kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u, kPhiloxW1 = 0xBB67AE85u;
constexpr uint32_t kStreamP = 1, kStreamE = 2, kStreamM = 3, kStreamN = 4;
constexpr int kMaxGrid = 16;

struct U4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * b) >> 32);
}

__host__ __device__ inline U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = kPhiloxM0 * c.x, hi0 = mulhi32(kPhiloxM0, c.x);
        const uint32_t lo1 = kPhiloxM1 * c.z, hi1 = mulhi32(kPhiloxM1, c.z);
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += kPhiloxW0;
        k1 += kPhiloxW1;
    }
    return c;
}

__device__ __forceinline__ U4 draw(uint32_t word, int64_t cw, uint32_t stream, uint32_t k0,
                                   uint32_t k1) {
    return philox4x32_10(U4{word, (uint32_t)cw, (uint32_t)((uint64_t)cw >> 32), stream}, k0, k1);
}

// uniform in (0, 1): 24 random bits, centred in their cell (never 0 or 1)
__device__ __forceinline__ float unit24(uint32_t u) {
    return ((float)(u >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// Box-Muller: two standard normals from two 32-bit draws (fp32, native log2 / sin / cos)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
    const float r = sqrtf(-2.0f * 0.6931471805599453f * __builtin_amdgcn_logf(unit24(a)));
    const float t = 6.283185307179586f * unit24(b);
    n0 = r * __cosf(t);
    n1 = r * __sinf(t);
}

struct ToricParams {
    uint32_t thr[kMaxGrid];     // Bernoulli threshold floor(p 2^32)
    double prior[kMaxGrid];     // log((1 - p) / p), computed on the host in double
    int np;
    uint32_t k0, k1;
    int64_t offset;
};

template <typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
sample_toric_kernel(GraphView g, ToricParams P, T* __restrict__ x, T* __restrict__ y, int64_t B,
                    int CW) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, N = g.N;
    const int tid = threadIdx.x;
    uint8_t* s_e = (uint8_t*)smem;                            // [CW][V] error bits
    int* s_p = (int*)(smem + (((size_t)CW * V + 15) & ~(size_t)15));   // [CW] grid index
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    for (int b = tid; b < nb; b += GNND_BLOCK) {
        const U4 r = draw(0, P.offset + b0 + b, kStreamP, P.k0, P.k1);
        s_p[b] = (int)mulhi32(r.x, (uint32_t)P.np);            // uniform over the grid
    }
    __syncthreads();
    const int VQ = (V + 3) >> 2;
    for (int i = tid; i < nb * VQ; i += GNND_BLOCK) {
        const int b = i / VQ, q = i - b * VQ;
        const int pi = GNND_DIDX(s_p[b], P.np, GNND_DBG_GRID);
        const U4 r = draw((uint32_t)q, P.offset + b0 + b, kStreamE, P.k0, P.k1);
        const uint32_t u[4] = {r.x, r.y, r.z, r.w};
        const uint32_t thr = P.thr[pi];
        const T prior = (T)P.prior[pi];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int v = 4 * q + j;
            if (v < V) {
                const uint8_t e = u[j] < thr ? 1 : 0;
                s_e[b * V + v] = e;
                y[(b0 + b) * V + v] = (T)e;
                x[(b0 + b) * N + v] = prior;
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < nb * C; i += GNND_BLOCK) {
        const int b = i / C, c = i - b * C;
        uint32_t par = 0;
        for (int k = g.chk_ptr[c], ke = g.chk_ptr[c + 1]; k < ke; ++k)
            par ^= s_e[b * V + GNND_DIDX((int)(g.edge_vc[g.chk_edge[k]] & 0xffffu), V, GNND_DBG_VAR)];
        x[(b0 + b) * N + V + c] = par ? T(-1) : T(1);
    }
}

struct AwgnParams {
    float sigma[kMaxGrid];      // sqrt(1 / 10^(SNR/10))
    float inv_var[kMaxGrid];    // 1 / sigma^2 in fp32  (post = 2 (y' * (1 / sigma^2)))
    int nsnr;
    int kw;                     // message words (0: constant codeword)
    uint32_t last_mask;         // valid bits of the last message word
    int bit;                    // constant codeword bit when kw == 0
    uint32_t k0, k1;
    int64_t offset;
};

template <typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
sample_awgn_kernel(int V, int C, AwgnParams P, const uint32_t* __restrict__ gen_cols,
                   T* __restrict__ x, T* __restrict__ y, int64_t B, int CW) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int N = V + C, KW = P.kw;
    const int tid = threadIdx.x;
    uint32_t* s_msg = (uint32_t*)smem;                        // [CW][KW] message words
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    const int KQ = (KW + 3) >> 2;
    for (int i = tid; i < nb * KQ; i += GNND_BLOCK) {
        const int b = i / KQ, q = i - b * KQ;
        const U4 r = draw((uint32_t)q, P.offset + b0 + b, kStreamM, P.k0, P.k1);
        const uint32_t u[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int w = 4 * q + j;
            if (w < KW) s_msg[b * KW + w] = w == KW - 1 ? (u[j] & P.last_mask) : u[j];
        }
    }
    __syncthreads();
    const int VQ = (V + 3) >> 2;
    for (int i = tid; i < nb * VQ; i += GNND_BLOCK) {
        const int b = i / VQ, q = i - b * VQ;
        const int64_t cw = P.offset + b0 + b;
        const int si = (int)(cw % P.nsnr);
        const float sigma = P.sigma[si], inv_var = P.inv_var[si];
        const U4 r = draw((uint32_t)q, cw, kStreamN, P.k0, P.k1);
        float n[4];
        box_muller(r.x, r.y, n[0], n[1]);
        box_muller(r.z, r.w, n[2], n[3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int v = 4 * q + j;
            if (v >= V) break;
            int c = P.bit;
            if (KW > 0) {
                uint32_t acc = 0;
                const uint32_t* gc = gen_cols + (size_t)v * KW;
                const uint32_t* m = s_msg + b * KW;
                for (int w = 0; w < KW; ++w) acc += __builtin_popcount(m[w] & gc[w]);
                c = (int)(acc & 1u);
            }
            const float yp = (1.0f - 2.0f * (float)c) + sigma * n[j];
            x[(b0 + b) * N + v] = (T)(2.0f * (yp * inv_var));
            y[(b0 + b) * V + v] = (T)c;
        }
    }
    for (int i = tid; i < nb * C; i += GNND_BLOCK) {
        const int b = i / C, c = i - b * C;
        x[(b0 + b) * N + V + c] = T(0);
    }
}

int tile_codewords(int N) {
    int cw = 4096 / (N > 0 ? N : 1);
    return cw < 1 ? 1 : (cw > 64 ? 64 : cw);
}

}  // namespace

GNND_DEBUG_TU(sample)

// host mirror of the generator (known-answer tests, tests/test_sample_cpu.py)
extern "C" void gnnd_philox4x32_10(const uint32_t* ctr4, const uint32_t* key2, uint32_t* out4) {
    const U4 r = philox4x32_10(U4{ctr4[0], ctr4[1], ctr4[2], ctr4[3]}, key2[0], key2[1]);
    out4[0] = r.x;
    out4[1] = r.y;
    out4[2] = r.z;
    out4[3] = r.w;
}

extern "C" int gnnd_sample_toric(const gnnd_graph* gr, int dtype, const double* h_p, int32_t n_p,
                                 uint64_t seed, int64_t offset, void* d_x, void* d_y,
                                 int64_t batch, void* stream) {
    if (!gr || !h_p || n_p < 1 || n_p > kMaxGrid || offset < 0 || batch < 0) return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_x || !d_y) return GNND_ERR_INVALID_ARG;
    ToricParams P{};
    for (int i = 0; i < n_p; ++i) {
        const double p = h_p[i];
        if (!(p > 0.0 && p < 1.0)) return GNND_ERR_INVALID_ARG;
        P.thr[i] = (uint32_t)(p * 4294967296.0);
        P.prior[i] = log((1.0 - p) / p);
    }
    P.np = n_p;
    P.k0 = (uint32_t)seed;
    P.k1 = (uint32_t)(seed >> 32);
    P.offset = offset;
    const GraphView& g = gr->view;
    const int cw = tile_codewords(g.N);
    const size_t lds = (((size_t)cw * g.V + 15) & ~(size_t)15) + (size_t)cw * 4;
    const int64_t blocks = (batch + cw - 1) / cw;
    if (blocks > 0x7fffffff || lds > 64 * 1024) return GNND_ERR_UNSUPPORTED;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        sample_toric_kernel<float><<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g, P, (float*)d_x, (float*)d_y, batch, cw);
    else
        sample_toric_kernel<double><<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g, P, (double*)d_x, (double*)d_y, batch, cw);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

extern "C" int gnnd_sample_awgn(const gnnd_graph* gr, int dtype, const double* h_snr_db,
                                int32_t n_snr, const uint32_t* d_gen_cols, int32_t k,
                                int32_t codeword_bit, uint64_t seed, int64_t offset, void* d_x,
                                void* d_y, int64_t batch, void* stream) {
    if (!gr || !h_snr_db || n_snr < 1 || n_snr > kMaxGrid || offset < 0 || batch < 0)
        return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64) return GNND_ERR_INVALID_ARG;
    if (d_gen_cols ? (k < 1 || k > 32 * 64) : (codeword_bit != 0 && codeword_bit != 1))
        return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_x || !d_y) return GNND_ERR_INVALID_ARG;
    AwgnParams P{};
    for (int i = 0; i < n_snr; ++i) {
        const double sigma = sqrt(1.0 / pow(10.0, h_snr_db[i] / 10.0));   // Gen_Data's Sigma
        P.sigma[i] = (float)sigma;
        P.inv_var[i] = 1.0f / ((float)sigma * (float)sigma);
    }
    P.nsnr = n_snr;
    P.kw = d_gen_cols ? (k + 31) / 32 : 0;
    P.last_mask = d_gen_cols && (k & 31) ? ((1u << (k & 31)) - 1u) : 0xffffffffu;
    P.bit = codeword_bit;
    P.k0 = (uint32_t)seed;
    P.k1 = (uint32_t)(seed >> 32);
    P.offset = offset;
    const GraphView& g = gr->view;
    const int cw = tile_codewords(g.N);
    const size_t lds = (size_t)cw * (P.kw > 0 ? P.kw : 1) * 4;
    const int64_t blocks = (batch + cw - 1) / cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        sample_awgn_kernel<float><<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g.V, g.C, P, d_gen_cols, (float*)d_x, (float*)d_y, batch, cw);
    else
        sample_awgn_kernel<double><<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g.V, g.C, P, d_gen_cols, (double*)d_x, (double*)d_y, batch, cw);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}
