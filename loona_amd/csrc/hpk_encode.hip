// hpk_encode.hip — gfx950 batched canonical Huffman encode (RFC 7541 §5.2; the H-bit branch
// crates/loona-hpack/src/encoder.rs:299-307 never takes — the reference has no encoder).
//
// v1: one lane per literal; the 257-entry code table sits in LDS; codes are packed MSB-first into
// a 64-bit accumulator, flushed a byte at a time, and the tail is padded with EOS MSBs (ones).
#include "hpk_device.h"

namespace {

struct EncodeArgs {
    const uint8_t* in_blob;
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_blob;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    const uint32_t* codes;  // [0,257): right-aligned code, [257,514): length
};

#define ENC_BLOCK 256

__global__ __launch_bounds__(ENC_BLOCK) void hpk_encode_kernel(EncodeArgs a) {
    __shared__ uint32_t s_code[256];
    __shared__ uint8_t s_len[256];
    if (threadIdx.x < 256) {
        s_code[threadIdx.x] = a.codes[threadIdx.x];
        s_len[threadIdx.x] = (uint8_t)a.codes[257 + threadIdx.x];
    }
    __syncthreads();
    for (uint32_t i = blockIdx.x * ENC_BLOCK + threadIdx.x; i < a.n; i += gridDim.x * ENC_BLOCK) {
        const uint32_t s = a.in_off[i], e = a.in_off[i + 1];
        const uint32_t o0 = a.out_off[i], ocap = a.out_off[i + 1] - o0;
        uint8_t* out = a.out_blob + o0;
        uint64_t acc = 0;
        int nb = 0;
        uint32_t o = 0;
        uint32_t st = HPK_OK;
        for (uint32_t p = s; p < e; ++p) {
            const uint32_t b = a.in_blob[p];
            acc = (acc << s_len[b]) | s_code[b];
            nb += s_len[b];
            while (nb >= 8) {
                nb -= 8;
                if (o >= ocap) { st = HPK_OUTPUT_OVERFLOW; break; }
                out[o++] = (uint8_t)(acc >> nb);
            }
            if (st) break;
        }
        if (!st && nb) {
            if (o >= ocap) st = HPK_OUTPUT_OVERFLOW;
            else out[o++] = (uint8_t)((acc << (8 - nb)) | (0xFFu >> nb));
        }
        a.out_len[i] = o;
        a.status[i] = (uint8_t)st;
    }
}


}  // namespace

int hpk_launch_encode(hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                      const uint32_t* out_off, uint32_t* out_len, uint8_t* status) {
    EncodeArgs a{in_blob, in_off, n, out_blob, out_off, out_len, status, c->d_codes};
    uint64_t blocks = ((uint64_t)n + ENC_BLOCK - 1) / ENC_BLOCK;
    const uint64_t max_blocks = (uint64_t)c->num_cu * 8;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(hpk_encode_kernel, dim3((uint32_t)blocks), dim3(ENC_BLOCK), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}
