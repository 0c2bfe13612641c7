// Direct 3x3 / 1x1 convolution for the depth predictor U-Nets' low-resolution levels on gfx950,
// exact fp32 MFMA.
//
// Semantics: torch.nn.functional.conv2d(x, w, bias, stride, padding = k // 2) on NCHW fp32 (the
// reference's nn.Conv2d layers in src/model/encoder/matching/ldm_unet/unet.py: ResBlock in/out
// convolutions unet.py:212-250, Downsample unet.py:140-170, Upsample unet.py:105-137, the ResBlock
// 1x1 skip unet.py:258-266), with two extensions that remove the glue around them:
//   * two input sources: x = cat([x1, x2], dim=1) read in place (the output blocks' skip concat);
//   * upsample = 1: x is first nearest-upsampled 2x (Upsample's F.interpolate) -- read in place.
//
// Why not MIOpen here: at 16^2..64^2 with 32..256 channels the fp32 convolutions are latency
// bound; MIOpen's NCHW kernels take 13-30 us each (~1.1 ms of the step over 56 launches), while
// the arithmetic is 9-600 MFLOP. This kernel spreads one 32 (cout) x 32 (pixel) output tile over
// `ksplit` waves of one workgroup (the reduction split over input-channel pairs), so even a 16^2
// layer fills hundreds of SIMDs.
//
// Implicit GEMM: D[co][px] = sum_k W[co][k] X[k][px], k = (tap, ci), one v_mfma_f32_32x32x2_f32
// per (tap, ci pair): A = the packed weights (one coalesced 256-B load per k-step, layout
// [co_tile][tap][ci/2][2][32], built once on the host), B = the input gathered at the tap's shifted
// pixel (32 consecutive pixels per lane half -> 128-B segments; padding lanes read a valid address
// and select 0). Each wave walks ci pairs w, w + ksplit, ... one batch (all 9 taps of 1-2 pairs, or
// 8-16 pairs of a 1x1) at a time with the next batch's loads in flight; the ksplit partial tiles are
// summed through LDS, the bias added, and the tile stored (lanes = consecutive pixels).
#include "common.h"
#include "prof.h"

namespace tsplat {
namespace conv {

constexpr int kMaxWaves = 16;

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct Args {
    const float* x1;
    const float* x2;
    const float* wp;    // packed weights [cot][taps][cin/2][2][32]
    const float* bias;  // [cout] or null
    const float* res;   // residual added to the output (y's layout) or null
    float* y;           // [n, cout, hout, wout] (NHWC: [n, hout, wout, cout])
    float* part;        // zsplit > 1: [tiles][zsplit][1024] partial tiles
    int* cnt;           // zsplit > 1: [tiles] arrival counters (zero between launches)
    int zsplit;         // workgroups per output tile (grid z)
    int c1, c2, cout, n;
    int hin, win;       // stored input size
    int hv, wv;         // virtual input size (2x when upsampling)
    int hout, wout;
    int npx;            // n * hout * wout
};

// The tile's ksplit (and zsplit) partial sums -> bias (+ residual) -> y. Every kernel here holds one
// 32 (cout) x 32 (pixel) tile per wave in the 32x32 MFMA accumulator layout (lane = pixel l & 31,
// register r = cout 8 (r >> 2) + 4 (l >> 5) + (r & 3)).
template <bool NHWC>
__device__ __forceinline__ void tile_epilogue(const Args& p, const floatx16& acc, float* sred) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ksplit = blockDim.x >> 6;
    const int cot = blockIdx.y;
    const int hwo = p.hout * p.wout;
    // sum the ksplit partial tiles
#pragma unroll
    for (int r = 0; r < 16; ++r) sred[(w * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
    const int tile = blockIdx.x + gridDim.x * blockIdx.y;
    if (p.zsplit > 1) {
        // this workgroup's partial tile -> workspace with agent-scope (write-through) stores, drained
        // by every wave; after the barrier ONE lane takes an arrival ticket with an agent-scope
        // RELEASE (cumulative over the workgroup's stores through the barrier: the HIP memory model's
        // publication, not only gfx9's write-through behaviour). The tile's last arriver: ONE
        // agent-scope acquire (its L1 may hold stale lines of the other partials), then plain loads
        // (cdna_hip_programming.md §5 "In-launch split-K reduction"; a __threadfence() in every
        // thread instead made the C2 step 5 % slower)
        typedef __attribute__((address_space(1))) unsigned gu32;
        unsigned* mine = reinterpret_cast<unsigned*>(p.part + ((size_t)tile * p.zsplit + blockIdx.z) * 1024);
        for (int idx = threadIdx.x; idx < 1024; idx += blockDim.x) {
            float s = 0.f;
            for (int k = 0; k < ksplit; ++k) s += sred[(k * 16 + (idx >> 6)) * 64 + (idx & 63)];
            __hip_atomic_store((gu32*)(mine + idx), __float_as_uint(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* flag = reinterpret_cast<int*>(sred + ksplit * 1024);  // one LDS word past the partials
        if (threadIdx.x == 0) {
            const int t = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const bool last = t == p.zsplit - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        const float* all = p.part + (size_t)tile * p.zsplit * 1024;
        for (int idx = threadIdx.x; idx < 1024; idx += blockDim.x) {
            float s = 0.f;
            for (int z = 0; z < p.zsplit; ++z) s += all[(size_t)z * 1024 + idx];
            sred[idx] = s;
        }
        __syncthreads();
    }
    const int nsum = p.zsplit > 1 ? 1 : ksplit;  // partial rows left in sred
    for (int idx = threadIdx.x; idx < 1024; idx += blockDim.x) {
        // NCHW: consecutive threads -> consecutive pixels; NHWC: -> consecutive output channels
        int r, l;
        if (NHWC) {
            const int col = idx & 31, pl = idx >> 5;
            r = ((col >> 3) << 2) | (col & 3);
            l = ((col >> 2) & 1) * 32 + pl;
        } else {
            r = idx >> 6;
            l = idx & 63;
        }
        float s = 0.f;
        for (int k = 0; k < nsum; ++k) s += sred[(k * 16 + r) * 64 + l];
        const int co = cot * 32 + 8 * (r >> 2) + 4 * (l >> 5) + (r & 3);
        const int q = blockIdx.x * 32 + (l & 31);
        if (co >= p.cout || q >= p.npx) continue;
        if (p.bias) s += p.bias[co];
        size_t o;
        if (NHWC) {
            o = (size_t)q * p.cout + co;
        } else {
            const int qn = q / hwo, qp = q - qn * hwo;
            o = ((size_t)qn * p.cout + co) * hwo + qp;
        }
        if (p.res) s += p.res[o];
        p.y[o] = s;
    }
}

// G = ci pairs per batch (all their taps): the loads of one batch are in flight while the previous
// batch's G * T MFMAs run, so a wave's time is ~ (its batches) x (memory latency) for these small
// layers -- larger G, fewer round trips.
// NHWC: input / output / residual channels-last ([n, h, w, c]; one source, no upsample) -- the DPT
// head's conv chain runs channels-last. RELU: ReLU applied to the input on load (the DPT
// ResidualConvUnit's activation before each convolution).
template <int KS, int S, int UP, int G, bool NHWC, bool RELU>
__global__ void __launch_bounds__(1024) conv_f32_kernel(Args p) {
    extern __shared__ float sred[];  // [ksplit][16][64]
    constexpr int T = KS * KS, PAD = KS / 2;
    constexpr int B = G * T;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ksplit = blockDim.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int cot = blockIdx.y;
    const int hwo = p.hout * p.wout, hwi = p.hin * p.win;
    const int px = blockIdx.x * 32 + c;
    const int pxc = min(px, p.npx - 1);
    const int nb = pxc / hwo, pix = pxc - nb * hwo;
    const int oy = pix / p.wout, ox = pix - oy * p.wout;
    const int cp_all = (p.c1 + p.c2) >> 1, cp1 = p.c1 >> 1;

    // per-tap input offset of this lane's pixel (0 = a valid address, masked, for padding)
    int off[T];
    unsigned vmask = 0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int ky = t / KS, kx = t - ky * KS;
        const int iy = oy * S + ky - PAD, ix = ox * S + kx - PAD;
        const bool v = px < p.npx && iy >= 0 && iy < p.hv && ix >= 0 && ix < p.wv;
        if (NHWC)
            off[t] = v ? (nb * hwi + iy * p.win + ix) * p.c1 : 0;
        else
            off[t] = v ? (UP ? (iy >> 1) * p.win + (ix >> 1) : iy * p.win + ix) : 0;
        vmask |= (unsigned)v << t;
    }
    const size_t wtap = (size_t)cp_all * 64;  // packed-weight stride between taps
    const float* wbase = p.wp + (size_t)cot * T * wtap + lane;
    // channel 2 cp + h of the concatenated input for this lane's image
    auto chan = [&](int cp) -> const float* {
        if (NHWC) return p.x1 + 2 * cp + h;
        return cp < cp1 ? p.x1 + ((size_t)nb * p.c1 + 2 * cp + h) * hwi
                        : p.x2 + ((size_t)nb * p.c2 + 2 * (cp - cp1) + h) * hwi;
    };
    // this wave's ci pairs: gw, gw + ksplit * zsplit, ... in batches of G (gw = its index over the
    // tile's zsplit workgroups)
    const int gw = blockIdx.z * ksplit + w, gstride = ksplit * p.zsplit;
    const int ncp = cp_all > gw ? (cp_all - gw + gstride - 1) / gstride : 0;
    const int nbatch = (ncp + G - 1) / G;
    // (called only when ncp > 0) every load is issued unconditionally from a clamped, valid
    // address and masked afterwards: a conditional load would become a branch with its own
    // s_waitcnt, serialising the batch's round trips
    auto load = [&](int bi, float* a, float* b) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int i = bi * G + g;
            const bool ok = i < ncp;
            const int cp = gw + min(i, ncp - 1) * gstride;
            const float* src = chan(cp);
            const float* wq = wbase + (size_t)cp * 64;
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const float av = wq[t * wtap];
                const float bv = RELU ? fmaxf(src[off[t]], 0.f) : src[off[t]];
                // masks applied to the bits (an AND with 0 or ~0: exactly +0 for a masked operand even
                // when the clamped address holds an Inf / NaN, where a multiply by 0 would give NaN),
                // so the loaded values are always used and the loads cannot sink into branches
                const unsigned ma = ok ? ~0u : 0u;
                const unsigned mb = (ok && ((vmask >> t) & 1)) ? ~0u : 0u;
                a[g * T + t] = __uint_as_float(__float_as_uint(av) & ma);
                b[g * T + t] = __uint_as_float(__float_as_uint(bv) & mb);
            }
        }
    };

    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (KS == 3) {
        // 3x3: one batch = G ci pairs x 9 taps, all of its loads issued before its MFMAs (one memory
        // round trip per batch); single-buffered so the 1024-thread workgroup stays within 128 VGPRs
        // (G = 4 is launched only when a wave has <= 4 pairs: one batch, no loop-carried state, so
        // the 72 operand registers fit next to the accumulator without spilling)
        const int nb = G == 4 ? min(nbatch, 1) : nbatch;
#pragma unroll 1
        for (int bi = 0; bi < nb; ++bi) {
            float ca[B], cb[B];
            load(bi, ca, cb);
            // keep the loads ahead of the MFMAs: left alone, the scheduler issues each load just before
            // its MFMA (a vmcnt(0) wait per k-step) to save registers
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < B; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[k], cb[k], acc, 0, 0, 0);
        }
    } else {
        // 1x1: 8-16 pairs per batch, the next batch's loads in flight during this batch's MFMAs
        float ca[B], cb[B], na[B], nbv[B];
        if (nbatch > 0) load(0, ca, cb);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
        for (int bi = 0; bi < nbatch; ++bi) {
            const bool more = bi + 1 < nbatch;
            if (more) load(bi + 1, na, nbv);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < B; ++k) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[k], cb[k], acc, 0, 0, 0);
            if (more) {
#pragma unroll
                for (int k = 0; k < B; ++k) {
                    ca[k] = na[k];
                    cb[k] = nbv[k];
                }
            }
        }
    }

    tile_epilogue<NHWC>(p, acc, sred);
}

// ---- split-bf16 ("bf16x3") form of the same convolution (the bf16x3 dense mode's precision: every
// product as hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation, x = hi + lo,
// <= ~3 * 2^-18 relative per product; the exact-fp32 32x32x2 MFMA above runs at 1/5.3 of its rate).
// The reduction is cut into units (tap t, 16-channel group g) -- one K = 16 MFMA triple each -- dealt
// to the tile's waves (and zsplit workgroups) round-robin; a wave loads NB units at once (per unit
// and lane: 8 channels of its pixel at the tap's shifted position, and the packed hi / lo weight
// fragments, two 16-B loads), splits the 8 values into hi / lo bf16 and issues the 3 MFMAs. Weights
// packed on the host as [co tile][tap][group][hi, lo][64 lanes][8] bf16 (lane l: cout 32 cot + (l & 31),
// channels 16 g + 8 (l >> 5) + j; zero past cin / cout). Epilogue as the fp32 kernel's.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((floatx2){a, b}, bf16x2));
}

template <int KS, int S, int UP, int NB>
__global__ void __launch_bounds__(1024) conv_x3_kernel(Args p) {
    extern __shared__ float sred[];  // [ksplit][16][64]
    constexpr int T = KS * KS, PAD = KS / 2;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ksplit = blockDim.x >> 6;
    const int h = lane >> 5;
    const int cot = blockIdx.y;
    const int hwo = p.hout * p.wout, hwi = p.hin * p.win;
    const int px = blockIdx.x * 32 + (lane & 31);
    const int pxc = min(px, p.npx - 1);
    const int nb = pxc / hwo, pix = pxc - nb * hwo;
    const int oy = pix / p.wout, ox = pix - oy * p.wout;
    const int ci = p.c1 + p.c2, ng = (ci + 15) >> 4;
    int off[T];
    unsigned vmask = 0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int ky = t / KS, kx = t - ky * KS;
        const int iy = oy * S + ky - PAD, ix = ox * S + kx - PAD;
        const bool v = px < p.npx && iy >= 0 && iy < p.hv && ix >= 0 && ix < p.wv;
        off[t] = v ? (UP ? (iy >> 1) * p.win + (ix >> 1) : iy * p.win + ix) : 0;
        vmask |= (unsigned)v << t;
    }
    const uint4* wbase = reinterpret_cast<const uint4*>(p.wp) + (size_t)cot * T * ng * 128 + lane;
    const int units = ng * T;
    const int gw = blockIdx.z * ksplit + w, gstride = ksplit * p.zsplit;
    const int nu = units > gw ? (units - gw + gstride - 1) / gstride : 0;
    const float* x1 = p.x1 + (size_t)nb * p.c1 * hwi;
    const float* x2 = p.x2 ? p.x2 + (size_t)nb * p.c2 * hwi : p.x1;

    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 1
    for (int b0 = 0; b0 < nu; b0 += NB) {
        float xv[NB][8];
        uint4 ah[NB], al[NB];
        // every load unconditional from a clamped, valid address, masked afterwards (a conditional
        // load becomes a branch with its own wait, serialising the batch's round trips)
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int i = b0 + k;
            const bool ok = i < nu;
            const int u = gw + min(i, nu - 1) * gstride;
            const int g = u / T, t = u - g * T;
            const uint4* wq = wbase + (size_t)(t * ng + g) * 128;
            const unsigned ma = ok ? ~0u : 0u;
            const uint4 a0 = wq[0], a1 = wq[64];
            ah[k] = make_uint4(a0.x & ma, a0.y & ma, a0.z & ma, a0.w & ma);
            al[k] = make_uint4(a1.x & ma, a1.y & ma, a1.z & ma, a1.w & ma);
            int o = 0;
            bool tv = false;
#pragma unroll
            for (int tt = 0; tt < T; ++tt)
                if (tt == t) {
                    o = off[tt];
                    tv = (vmask >> tt) & 1;
                }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int ch = 16 * g + 8 * h + j;
                const int cc = min(ch, ci - 1);
                const float* src = cc < p.c1 ? x1 + (size_t)cc * hwi : x2 + (size_t)(cc - p.c1) * hwi;
                const float v = src[o];
                const unsigned mb = (ok && tv && ch < ci) ? ~0u : 0u;
                xv[k][j] = __uint_as_float(__float_as_uint(v) & mb);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            uint32_t hi[4], lo[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float a = xv[k][2 * q], b = xv[k][2 * q + 1];
                hi[q] = pack_bf16(a, b);
                const float ah_ = __uint_as_float(hi[q] << 16), bh_ = __uint_as_float(hi[q] & 0xffff0000u);
                lo[q] = pack_bf16(a - ah_, b - bh_);
            }
            const bf16x8 bh = __builtin_bit_cast(bf16x8, make_uint4(hi[0], hi[1], hi[2], hi[3]));
            const bf16x8 bl = __builtin_bit_cast(bf16x8, make_uint4(lo[0], lo[1], lo[2], lo[3]));
            const bf16x8 wh = __builtin_bit_cast(bf16x8, ah[k]), wl = __builtin_bit_cast(bf16x8, al[k]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bh, acc, 0, 0, 0);
        }
    }
    tile_epilogue<false>(p, acc, sred);
}

}  // namespace conv
}  // namespace tsplat

extern "C" int tsplat_conv2d_f32_zsplit_fwd(const float* x1, int32_t c1, const float* x2, int32_t c2,
                                            const float* w_packed, const float* bias, float* y, int32_t batch,
                                            int32_t height, int32_t width, int32_t c_out, int32_t ksize,
                                            int32_t stride, int32_t upsample, int32_t ksplit, int32_t zsplit,
                                            float* partials, int32_t* counters, void* stream_) {
    using namespace tsplat::conv;
    if (!x1 || !w_packed || !y || batch <= 0 || height <= 0 || width <= 0 || c_out <= 0) return TSPLAT_EINVAL;
    if (zsplit < 1 || zsplit > 64 || (zsplit > 1 && (!partials || !counters))) return TSPLAT_EINVAL;
    if (c1 <= 0 || (c1 & 1) || c2 < 0 || (c2 & 1) || (c2 > 0 && !x2)) return TSPLAT_EINVAL;
    if (!(ksize == 1 || ksize == 3) || !(stride == 1 || stride == 2) || !(upsample == 0 || upsample == 1))
        return TSPLAT_EINVAL;
    if (ksplit < 1 || ksplit > kMaxWaves) return TSPLAT_EINVAL;
    Args p{};
    p.zsplit = zsplit;
    p.part = partials;
    p.cnt = counters;
    p.x1 = x1;
    p.x2 = x2;
    p.wp = w_packed;
    p.bias = bias;
    p.y = y;
    p.c1 = c1;
    p.c2 = c2;
    p.cout = c_out;
    p.n = batch;
    p.hin = height;
    p.win = width;
    p.hv = upsample ? 2 * height : height;
    p.wv = upsample ? 2 * width : width;
    const int pad = ksize / 2;
    p.hout = (p.hv + 2 * pad - ksize) / stride + 1;
    p.wout = (p.wv + 2 * pad - ksize) / stride + 1;
    if (p.hout <= 0 || p.wout <= 0) return TSPLAT_EINVAL;
    const int64_t npx = (int64_t)batch * p.hout * p.wout;
    const int64_t in_elems = (int64_t)batch * (c1 > c2 ? c1 : c2) * height * width;
    if (npx >= (1ll << 31) || in_elems >= (1ll << 31)) return TSPLAT_EINVAL;
    p.npx = (int)npx;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)((npx + 31) / 32), (unsigned)((c_out + 31) / 32), (unsigned)zsplit);
    const dim3 block(64 * ksplit);
    const size_t lds = (size_t)ksplit * 16 * 64 * sizeof(float) + 16;  // + the last-arriver flag
    TSPLAT_PROF_BEGIN(tsplat::prof::kConv, stream);
#define TSPLAT_CONV_LAUNCH(KS, S, UP, G) \
    hipLaunchKernelGGL((conv_f32_kernel<KS, S, UP, G, false, false>), grid, block, lds, stream, p)
    // ci pairs per batch: 3x3 -> all of a wave's 3-4 pairs in one batch, else 2 (1 if it has 1);
    // 1x1 -> 16 once a wave has that many, else 8
    const int per_wave = ((c1 + c2) / 2 + ksplit * zsplit - 1) / (ksplit * zsplit);
    const bool wide = per_wave >= (ksize == 3 ? 2 : 16);
    const bool one = ksize == 3 && per_wave >= 3 && per_wave <= 4;
    if (ksize == 3 && stride == 1 && !upsample) {
        if (one) TSPLAT_CONV_LAUNCH(3, 1, 0, 4); else if (wide) TSPLAT_CONV_LAUNCH(3, 1, 0, 2); else TSPLAT_CONV_LAUNCH(3, 1, 0, 1);
    } else if (ksize == 3 && stride == 2 && !upsample) {
        if (one) TSPLAT_CONV_LAUNCH(3, 2, 0, 4); else if (wide) TSPLAT_CONV_LAUNCH(3, 2, 0, 2); else TSPLAT_CONV_LAUNCH(3, 2, 0, 1);
    } else if (ksize == 3 && stride == 1 && upsample) {
        if (one) TSPLAT_CONV_LAUNCH(3, 1, 1, 4); else if (wide) TSPLAT_CONV_LAUNCH(3, 1, 1, 2); else TSPLAT_CONV_LAUNCH(3, 1, 1, 1);
    } else if (ksize == 1 && stride == 1 && !upsample) {
        if (wide) TSPLAT_CONV_LAUNCH(1, 1, 0, 16); else TSPLAT_CONV_LAUNCH(1, 1, 0, 8);
    } else if (ksize == 1 && stride == 2 && !upsample) {  // the CNN's strided 1x1 shortcut
        TSPLAT_CONV_LAUNCH(1, 2, 0, 8);
    } else {
        return TSPLAT_EINVAL;
    }
#undef TSPLAT_CONV_LAUNCH
    TSPLAT_PROF_END(tsplat::prof::kConv, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_conv2d_f32_fwd(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* w_packed,
                                     const float* bias, float* y, int32_t batch, int32_t height, int32_t width,
                                     int32_t c_out, int32_t ksize, int32_t stride, int32_t upsample, int32_t ksplit,
                                     void* stream_) {
    return tsplat_conv2d_f32_zsplit_fwd(x1, c1, x2, c2, w_packed, bias, y, batch, height, width, c_out, ksize, stride,
                                        upsample, ksplit, 1, nullptr, nullptr, stream_);
}

extern "C" int tsplat_conv2d_f32_nhwc_fwd(const float* x, int32_t c_in, const float* w_packed, const float* bias,
                                          const float* residual, float* y, int32_t batch, int32_t height,
                                          int32_t width, int32_t c_out, int32_t ksize, int32_t relu_in,
                                          int32_t ksplit, void* stream_) {
    using namespace tsplat::conv;
    if (!x || !w_packed || !y || batch <= 0 || height <= 0 || width <= 0 || c_out <= 0) return TSPLAT_EINVAL;
    if (c_in <= 0 || (c_in & 1) || !(ksize == 1 || ksize == 3) || ksplit < 1 || ksplit > kMaxWaves)
        return TSPLAT_EINVAL;
    const int64_t elems = (int64_t)batch * height * width * (c_in > c_out ? c_in : c_out);
    if (elems >= (1ll << 31)) return TSPLAT_EINVAL;
    Args p{};
    p.x1 = x;
    p.wp = w_packed;
    p.bias = bias;
    p.res = residual;
    p.y = y;
    p.c1 = c_in;
    p.cout = c_out;
    p.n = batch;
    p.hin = p.hv = p.hout = height;
    p.win = p.wv = p.wout = width;
    p.npx = batch * height * width;
    p.zsplit = 1;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)((p.npx + 31) / 32), (unsigned)((c_out + 31) / 32));
    const dim3 block(64 * ksplit);
    const size_t lds = (size_t)ksplit * 16 * 64 * sizeof(float);
    const int per_wave = (c_in / 2 + ksplit - 1) / ksplit;
    const bool wide = per_wave >= (ksize == 3 ? 2 : 16);
    TSPLAT_PROF_BEGIN(tsplat::prof::kConv, stream);
#define TSPLAT_CONV_LAUNCH(KS, G, RELU) \
    hipLaunchKernelGGL((conv_f32_kernel<KS, 1, 0, G, true, RELU>), grid, block, lds, stream, p)
    if (ksize == 3) {
        if (relu_in) {
            if (wide) TSPLAT_CONV_LAUNCH(3, 2, true); else TSPLAT_CONV_LAUNCH(3, 1, true);
        } else {
            if (wide) TSPLAT_CONV_LAUNCH(3, 2, false); else TSPLAT_CONV_LAUNCH(3, 1, false);
        }
    } else {
        if (relu_in) {
            if (wide) TSPLAT_CONV_LAUNCH(1, 16, true); else TSPLAT_CONV_LAUNCH(1, 8, true);
        } else {
            if (wide) TSPLAT_CONV_LAUNCH(1, 16, false); else TSPLAT_CONV_LAUNCH(1, 8, false);
        }
    }
#undef TSPLAT_CONV_LAUNCH
    TSPLAT_PROF_END(tsplat::prof::kConv, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_conv2d_bf16x3_fwd(const float* x1, int32_t c1, const float* x2, int32_t c2,
                                        const void* w_packed, const float* bias, float* y, int32_t batch,
                                        int32_t height, int32_t width, int32_t c_out, int32_t ksize, int32_t stride,
                                        int32_t upsample, int32_t ksplit, int32_t zsplit, float* partials,
                                        int32_t* counters, void* stream_) {
    using namespace tsplat::conv;
    if (!x1 || !w_packed || !y || batch <= 0 || height <= 0 || width <= 0 || c_out <= 0) return TSPLAT_EINVAL;
    if (zsplit < 1 || zsplit > 64 || (zsplit > 1 && (!partials || !counters))) return TSPLAT_EINVAL;
    if (c1 <= 0 || c2 < 0 || (c2 > 0 && !x2)) return TSPLAT_EINVAL;
    if (!(ksize == 1 || ksize == 3) || !(stride == 1 || stride == 2) || !(upsample == 0 || upsample == 1) ||
        (upsample && stride != 1))
        return TSPLAT_EINVAL;
    if (ksplit < 1 || ksplit > kMaxWaves) return TSPLAT_EINVAL;
    Args p{};
    p.zsplit = zsplit;
    p.part = partials;
    p.cnt = counters;
    p.x1 = x1;
    p.x2 = c2 > 0 ? x2 : nullptr;
    p.wp = (const float*)w_packed;
    p.bias = bias;
    p.y = y;
    p.c1 = c1;
    p.c2 = c2;
    p.cout = c_out;
    p.n = batch;
    p.hin = height;
    p.win = width;
    p.hv = upsample ? 2 * height : height;
    p.wv = upsample ? 2 * width : width;
    const int pad = ksize / 2;
    p.hout = (p.hv + 2 * pad - ksize) / stride + 1;
    p.wout = (p.wv + 2 * pad - ksize) / stride + 1;
    if (p.hout <= 0 || p.wout <= 0) return TSPLAT_EINVAL;
    const int64_t npx = (int64_t)batch * p.hout * p.wout;
    const int64_t in_elems = (int64_t)batch * (c1 > c2 ? c1 : c2) * height * width;
    if (npx >= (1ll << 31) || in_elems >= (1ll << 31)) return TSPLAT_EINVAL;
    p.npx = (int)npx;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)((npx + 31) / 32), (unsigned)((c_out + 31) / 32), (unsigned)zsplit);
    const dim3 block(64 * ksplit);
    const size_t lds = (size_t)ksplit * 16 * 64 * sizeof(float) + 16;
    // units per wave: one batch when a wave has up to 4, else batches of 2 (batches of 4 measured up
    // to 2x slower there: 120 VGPRs, profiles/r5/conv_x3/census_x3b.log)
    const int units = (c1 + c2 + 15) / 16 * ksize * ksize;
    const int per_wave = (units + ksplit * zsplit - 1) / (ksplit * zsplit);
    const int nb = per_wave <= 4 ? per_wave : 2;
    TSPLAT_PROF_BEGIN(tsplat::prof::kConv, stream);
#define TSPLAT_X3_LAUNCH(KS, S, UP)                                                                       \
    do {                                                                                                  \
        if (nb == 1) hipLaunchKernelGGL((conv_x3_kernel<KS, S, UP, 1>), grid, block, lds, stream, p);     \
        else if (nb == 3) hipLaunchKernelGGL((conv_x3_kernel<KS, S, UP, 3>), grid, block, lds, stream, p); \
        else if (nb == 4) hipLaunchKernelGGL((conv_x3_kernel<KS, S, UP, 4>), grid, block, lds, stream, p); \
        else hipLaunchKernelGGL((conv_x3_kernel<KS, S, UP, 2>), grid, block, lds, stream, p);             \
    } while (0)
    if (ksize == 3 && stride == 1 && !upsample) TSPLAT_X3_LAUNCH(3, 1, 0);
    else if (ksize == 3 && stride == 2) TSPLAT_X3_LAUNCH(3, 2, 0);
    else if (ksize == 3) TSPLAT_X3_LAUNCH(3, 1, 1);
    else if (stride == 1) TSPLAT_X3_LAUNCH(1, 1, 0);
    else TSPLAT_X3_LAUNCH(1, 2, 0);
#undef TSPLAT_X3_LAUNCH
    TSPLAT_PROF_END(tsplat::prof::kConv, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
