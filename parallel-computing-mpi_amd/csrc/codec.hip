// codec.hip -- lossless delta coding of sorted key runs for the compare-split
// exchange over xGMI (gfx950).
//
// The keys a rank sends in one compare-split stage (psort.cc:116-164: the
// reference ships the whole block with MPI_Sendrecv) are a sorted run, so
// consecutive differences are small: 2^27 uniform u32 keys have a mean gap of
// 32.  The run is cut into blocks of CB keys; a block is stored as its first
// key (base) and its CB-1 gaps packed at the block's own bit width w (the
// width of its largest gap), "frame of reference" style.  Decoding is a
// block-wide prefix sum.  Every block decodes independently, so encode and
// decode are single HBM-streaming passes.
//
// Stream (u32 words): nblk headers of 4 words {base lo, base hi, payload
// offset (words, from the stream start), width}, then the payloads.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace misort {
namespace {

constexpr int CB = 1024, CT = 256, CI = CB / CT;  // keys per block, threads, keys per thread

__device__ __forceinline__ int width_of(uint64_t d) { return d ? 64 - __builtin_clzll(d) : 0; }

// Per block: payload words for its gaps at the block's width.  (Lane-strided
// loads of 4 consecutive keys; measured faster here than coalesced loads with a
// cross-lane predecessor, and than packing through LDS atomics.)
template <typename K>
__global__ __launch_bounds__(CT) void k_codec_width(const K* __restrict__ keys, int64_t n,
                                                    uint32_t* __restrict__ words, uint8_t* __restrict__ wid) {
    __shared__ uint64_t red[CT / 64];
    const int64_t b = blockIdx.x, k0 = b * CB;
    const int t = threadIdx.x;
    uint64_t mx = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
        const int64_t j = k0 + t * CI + i;  // gap: key j minus key j-1
        if (j > k0 && j < n) mx = max(mx, (uint64_t)(keys[j] - keys[j - 1]));
    }
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, o));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    if (t == 0) {
        for (int i = 1; i < CT / 64; ++i) mx = max(mx, red[i]);
        const int w = width_of(mx);
        const int64_t cnt = n - k0 < CB ? n - k0 : CB;
        words[b] = (uint32_t)(((cnt - 1) * w + 31) >> 5);
        wid[b] = (uint8_t)w;
    }
}

template <typename K>
__global__ __launch_bounds__(CT) void k_codec_pack(const K* __restrict__ keys, int64_t n, int64_t nblk,
                                                   const uint32_t* __restrict__ off, const uint8_t* __restrict__ wid,
                                                   uint32_t* __restrict__ out) {
    __shared__ uint64_t gap[CB];
    const int64_t b = blockIdx.x, k0 = b * CB;
    const int t = threadIdx.x;
    const int64_t cnt = n - k0 < CB ? n - k0 : CB;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
        const int j = t * CI + i;  // gap j: key k0+j+1 minus key k0+j
        gap[j] = (j + 1 < cnt) ? (uint64_t)(keys[k0 + j + 1] - keys[k0 + j]) : 0;
    }
    __syncthreads();
    const int w = wid[b];
    const uint32_t base_w = (uint32_t)(4 * nblk) + off[b];
    const int nw = (int)(((cnt - 1) * w + 31) >> 5);
    if (t == 0) {
        const uint64_t base = (uint64_t)keys[k0];
        uint32_t* h = out + 4 * b;
        h[0] = (uint32_t)base;
        h[1] = (uint32_t)(base >> 32);
        h[2] = base_w;
        h[3] = (uint32_t)w;
    }
    for (int q = t; q < nw; q += CT) {
        // fields j overlapping bits [32q, 32q+32)
        const int64_t lo = (int64_t)q * 32;
        uint32_t v = 0;
        for (int64_t j = lo / w; j * w < lo + 32 && j < cnt - 1; ++j) {
            const int64_t sh = j * w - lo;  // field start relative to the word (may be < 0)
            const uint64_t f = gap[j];
            v |= sh >= 0 ? (uint32_t)(f << sh) : (uint32_t)(f >> (-sh));
        }
        out[base_w + q] = v;
    }
}

__global__ void k_codec_total(const uint32_t* off, const uint32_t* words, int64_t nb, uint32_t* total) {
    *total = (uint32_t)(4 * nb) + off[nb - 1] + words[nb - 1];
}

// Lane t rebuilds keys 4t..4t+3 of its block: key p = base + the gaps before
// it, so the lane decodes gaps 4t-1..4t+2, a wave scan (cross-lane shuffles) and one
// LDS step across the 4 waves give the prefix, and the 4 keys leave as one
// 16-byte (u32) or two (u64) vector stores.
template <typename K>
__global__ __launch_bounds__(CT) void k_codec_unpack(const uint32_t* __restrict__ in, int64_t n,
                                                     K* __restrict__ keys) {
    static_assert(CI == 4, "one 4-key run per lane");
    __shared__ uint64_t wsum[CT / 64];
    const int64_t b = blockIdx.x, k0 = b * CB;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t cnt = n - k0 < CB ? n - k0 : CB;
    const uint32_t* h = in + 4 * b;
    const uint64_t base = (uint64_t)h[0] | ((uint64_t)h[1] << 32);
    const uint32_t pw = h[2];
    const int w = (int)h[3];
    const uint64_t mask = w >= 64 ? ~0ull : ((1ull << w) - 1);
    uint64_t g[CI], s = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
        const int64_t j = (int64_t)t * CI + i - 1;  // the gap before key 4t+i
        uint64_t f = 0;
        if (w && j >= 0 && j + 1 < cnt) {
            const int64_t bit = j * w;
            const uint32_t* p = in + pw + (bit >> 5);
            const int sh = (int)(bit & 31);
            const uint64_t lo = (uint64_t)p[0] | ((uint64_t)(sh + w > 32 ? p[1] : 0) << 32);
            f = lo >> sh;
            if (sh + w > 64) f |= (uint64_t)p[2] << (64 - sh);
            f &= mask;
        }
        s += f;
        g[i] = s;  // inclusive prefix within the lane
    }
    uint64_t x = s;  // inclusive scan of the lane totals over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t pre = x - s;
    for (int v = 0; v < wv; ++v) pre += wsum[v];
    K r[CI];
#pragma unroll
    for (int i = 0; i < CI; ++i) r[i] = (K)(base + pre + g[i]);
    const int64_t p0 = k0 + (int64_t)t * CI;
    if ((int64_t)t * CI + CI <= cnt && !((uintptr_t)(keys + p0) & 15)) {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        v4* dst = reinterpret_cast<v4*>(keys + p0);
        if constexpr (sizeof(K) == 4) {
            dst[0] = v4{(uint32_t)r[0], (uint32_t)r[1], (uint32_t)r[2], (uint32_t)r[3]};
        } else {
            dst[0] = v4{(uint32_t)r[0], (uint32_t)((uint64_t)r[0] >> 32), (uint32_t)r[1],
                        (uint32_t)((uint64_t)r[1] >> 32)};
            dst[1] = v4{(uint32_t)r[2], (uint32_t)((uint64_t)r[2] >> 32), (uint32_t)r[3],
                        (uint32_t)((uint64_t)r[3] >> 32)};
        }
    } else {
#pragma unroll
        for (int i = 0; i < CI; ++i)
            if ((int64_t)t * CI + i < cnt) keys[p0 + i] = r[i];
    }
}

}  // namespace

int64_t codec_blocks(int64_t n) { return (n + CB - 1) / CB; }

size_t codec_scratch_bytes(int64_t n) {
    const int64_t nb = codec_blocks(n) > 0 ? codec_blocks(n) : 1;
    size_t tmp = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)nb);
    return (size_t)nb * (2 * sizeof(uint32_t) + 1) + 512 + tmp;
}

int64_t codec_max_words(int64_t n, int key_bytes) {
    return 4 * codec_blocks(n) + (n * key_bytes * 8 + 31) / 32 + codec_blocks(n);
}

template <typename K>
hipError_t codec_encode(const K* keys, int64_t n, uint32_t* out, void* scratch, size_t scratch_bytes,
                        uint32_t* d_total, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = codec_blocks(n);
    char* p = (char*)scratch;
    uint32_t* words = (uint32_t*)p;
    uint32_t* off = words + nb;
    uint8_t* wid = (uint8_t*)(off + nb);
    void* tmp = (void*)(((uintptr_t)(wid + nb) + 255) & ~(uintptr_t)255);
    size_t tmp_bytes = scratch_bytes - (size_t)((char*)tmp - p);
    k_codec_width<K><<<(unsigned)nb, CT, 0, s>>>(keys, n, words, wid);
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, words, off, (int)nb, s);
    if (e != hipSuccess) return e;
    k_codec_pack<K><<<(unsigned)nb, CT, 0, s>>>(keys, n, nb, off, wid, out);
    k_codec_total<<<1, 1, 0, s>>>(off, words, nb, d_total);
    return hipGetLastError();
}

template <typename K>
hipError_t codec_decode(const uint32_t* in, int64_t n, K* keys, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_codec_unpack<K><<<(unsigned)codec_blocks(n), CT, 0, s>>>(in, n, keys);
    return hipGetLastError();
}

template hipError_t codec_encode<uint32_t>(const uint32_t*, int64_t, uint32_t*, void*, size_t, uint32_t*,
                                           hipStream_t);
template hipError_t codec_encode<uint64_t>(const uint64_t*, int64_t, uint32_t*, void*, size_t, uint32_t*,
                                           hipStream_t);
template hipError_t codec_decode<uint32_t>(const uint32_t*, int64_t, uint32_t*, hipStream_t);
template hipError_t codec_decode<uint64_t>(const uint32_t*, int64_t, uint64_t*, hipStream_t);

}  // namespace misort
