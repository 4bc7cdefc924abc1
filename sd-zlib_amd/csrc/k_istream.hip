// k_istream.hip -- incremental inflate (Inflater.append across calls, sd-inflate.ts:87-153):
// the state slab's reset and the per-call input staging.
//
// Between calls a stream keeps, in device memory: its decoder state (DSave: bit position,
// block mode, Huffman trees -- inflate.ts:79-95, infblocks.ts:45-50, infcodes.ts:35-55),
// its resolve state (RSave: running checksum, output and input totals), the last 32 KiB of
// output (the LZ77 window) and the input bytes of the unit it could not finish (a header,
// a block header, a symbol: the bits the reference keeps in its bit buffer).  A call
// stages carry + new chunk contiguously so that the decoder reads one input run, exactly
// as in the one-shot path.
#include "inflate_state.h"

namespace sdz {

__global__ void k_istate_reset(uint8_t* dsave, uint8_t* rsave, uint32_t n) {
    const uint32_t sid = blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= n) return;
    DSave* S = (DSave*)dsave + sid;
    RSave* R = (RSave*)rsave + sid;
    S->mode = LM_INIT; S->status = SDZ_OK; S->zmsg = 0; S->stall = 0;
    S->bitpos = 0; S->pos = 0; S->full = 0; S->ntok = 0; S->litw = 0; S->nlit = 0;
    S->container = SDZ_CONTAINER_RAW; S->stored_ck = 0; S->stored_size = 0; S->mtime = 0;
    S->name_off = 0; S->name_len = 0; S->dict_used = 0;
    R->pos = 0; R->s1 = 0; R->s2 = 0; R->ck = 0; R->hist = 0;
    R->total = 0; R->in_base = 0; R->a1 = 1; R->a2 = 0; R->crc = 0; R->carry_len = 0;
    R->abase = 0; R->a1s = 1; R->a2s = 0;
}

// one block per stream: stage = carry ++ chunk; a finished stream given more bytes reports
// them (the reference's append() throws "bad input data" there, sd-inflate.ts:130-132)
// staging slot of stream i: SDZ_INFLATE_CARRY + in_len + 64 bytes (readable slack for the
// decoder's 16-byte loads), 256-aligned; st_off = exclusive prefix sums, one workgroup
#define SG_THREADS 1024
__device__ __forceinline__ uint64_t stage_slot(uint64_t len) { return (SDZ_INFLATE_CARRY + len + 64 + 255) & ~255ull; }
__global__ __launch_bounds__(SG_THREADS) void k_stage_slots(const uint64_t* in_len, uint32_t n, uint64_t* st_off) {
    __shared__ uint64_t part[SG_THREADS];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + SG_THREADS - 1) / SG_THREADS;
    const uint32_t b = t * per < n ? t * per : n, e = b + per < n ? b + per : n;
    uint64_t sum = 0;
    for (uint32_t i = b; i < e; ++i) sum += stage_slot(in_len[i]);
    part[t] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < SG_THREADS; o <<= 1) {      // inclusive scan of the thread sums
        const uint64_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0;
    for (uint32_t i = b; i < e; ++i) { st_off[i] = run; run += stage_slot(in_len[i]); }
}

__global__ __launch_bounds__(256) void k_istate_stage(InflateArgs A, const uint8_t* in, const uint64_t* in_off,
                                                      const uint64_t* in_len, uint8_t* stage,
                                                      uint64_t* st_off, uint64_t* st_len) {
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    DSave* S = (DSave*)A.dsave + sid;
    RSave* R = (RSave*)A.rsave + sid;
    const uint32_t nc = R->carry_len;
    const uint64_t nl = in_len[sid];
    uint8_t* dst = stage + st_off[sid];
    const uint8_t* carry = A.carry + (uint64_t)sid * SDZ_INFLATE_CARRY;
    const uint8_t* src = in + in_off[sid];
    for (uint32_t k = threadIdx.x; k < nc; k += blockDim.x) dst[k] = carry[k];
    dst += nc;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const uint64_t nv = nl >> 4;
        for (uint64_t k = threadIdx.x; k < nv; k += blockDim.x) ((uint4*)dst)[k] = ((const uint4*)src)[k];
        for (uint64_t k = (nv << 4) + threadIdx.x; k < nl; k += blockDim.x) dst[k] = src[k];
    } else {
        for (uint64_t k = threadIdx.x; k < nl; k += blockDim.x) dst[k] = src[k];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    st_len[sid] = nc + nl;                         // R->carry_len stays: the staged input's carried head
    // a call that does not continue an append stopped at out_cap starts a new append():
    // its output chunks (and the running adler32's NMAX grid) start here
    if (!(S->stall == 2 && S->mode != LM_DONE)) { R->abase = R->total; R->a1s = R->a1; R->a2s = R->a2; }
    if (S->mode == LM_DONE && nl > 0 && S->status == SDZ_OK) S->status = SDZ_TRAILING;
}

void launch_istate_reset(uint8_t* dsave, uint8_t* rsave, uint32_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_istate_reset, dim3((n + 255) / 256), dim3(256), 0, s, dsave, rsave, n);
}

void launch_istate_stage(const InflateArgs& a, const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                         uint8_t* stage, uint64_t* st_off, uint64_t* st_len, hipStream_t s) {
    if (!a.n) return;
    hipLaunchKernelGGL(k_stage_slots, dim3(1), dim3(SG_THREADS), 0, s, in_len, a.n, st_off);
    hipLaunchKernelGGL(k_istate_stage, dim3(a.n), dim3(256), 0, s, a, in, in_off, in_len, stage, st_off, st_len);
}

}  // namespace sdz
