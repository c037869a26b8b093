// s2c_bodies.hip — FASTA body assembly on the device (:394-418): the tiles' body slots of
// the output buffer compacted into one contiguous byte array in [threshold][tile] order.
//
// The tile kernels write each (threshold, tile) body into a static slot of `out`
// (s2c_dev.out: t·(F·padded_len + n_cols) + F·a + cb0) — no scan between tiles.  A body is
// shorter than its slot wherever an insertion column voted '-' (:370-385) or the tile has no
// columns' worth of insertions, so the slots are not contiguous; this kernel gathers them so
// a single D2H copy (one GPU) or one collective (a multi-GPU rank's bodies, shard.py) moves
// exactly the body bytes.  It is HBM-bound byte movement: one workgroup per block, 16-byte
// stores wherever the destination is aligned (a C5 tile's 1,024-byte body is 64 of them).
#include "s2c_common.h"

namespace s2c {
namespace {

constexpr int BWG = 256;

// block i: dst[offs[i], offs[i+1]) = out[starts[i], starts[i] + offs[i+1] - offs[i]); bytes
// past out_len are not read (the host's starts are checked there, this only guards)
__global__ __launch_bounds__(BWG) void k_bodies(const uint8_t *__restrict__ out, uint64_t out_len,
                                                 const int64_t *__restrict__ starts, const int64_t *__restrict__ offs,
                                                 uint64_t n, uint8_t *__restrict__ dst) {
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t d0 = offs[i], d1 = offs[i + 1], s0 = starts[i];
        if (d1 <= d0 || s0 < 0) continue;
        const uint64_t len = (uint64_t)(d1 - d0);
        if ((uint64_t)s0 > out_len || len > out_len - (uint64_t)s0) continue;
        const uint8_t *src = out + s0;
        uint8_t *d = dst + d0;
        // head bytes up to the destination's 16-byte boundary, then 16-byte destination
        // words assembled from byte loads (the source is rarely aligned with it), then the tail
        const uint64_t head = min<uint64_t>(len, (16u - ((uintptr_t)d & 15u)) & 15u);
        for (uint64_t k = threadIdx.x; k < head; k += BWG) d[k] = src[k];
        const uint64_t nv = (len - head) / 16;
        for (uint64_t v = threadIdx.x; v < nv; v += BWG) {
            const uint8_t *s = src + head + 16 * v;
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                w[j] = (uint32_t)s[4 * j] | (uint32_t)s[4 * j + 1] << 8 | (uint32_t)s[4 * j + 2] << 16 |
                       (uint32_t)s[4 * j + 3] << 24;
            *(uint4 *)(d + head + 16 * v) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        for (uint64_t k = head + 16 * nv + threadIdx.x; k < len; k += BWG) d[k] = src[k];
    }
}

}  // namespace
}  // namespace s2c

extern "C" int s2c_gather_bodies_dev(const uint8_t *out, int64_t out_len, const int64_t *starts, const int64_t *offs,
                                     int64_t n, uint8_t *dst, void *stream) {
    using namespace s2c;
    if (n < 0 || out_len < 0) return s2c_set_error(S2C_ERR_ARG, "bad body gather sizes");
    if (n == 0) return S2C_OK;
    if (!out || !starts || !offs || !dst) return s2c_set_error(S2C_ERR_ARG, "NULL body gather buffer");
    const unsigned grid = (unsigned)std::min<int64_t>(n, 8 * 256 * 4);   // ≥ 8 workgroups per CU in flight
    k_bodies<<<grid, BWG, 0, (hipStream_t)stream>>>(out, (uint64_t)out_len, starts, offs, (uint64_t)n, dst);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? S2C_OK : s2c_set_error(S2C_ERR_HIP, std::string("k_bodies: ") + hipGetErrorString(e));
}
