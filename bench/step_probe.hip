// step_probe.hip — development probe (not part of the product): the latency of one lane-walk body
// step (lit12_body, the wave kernel's LUT3 form) in isolation, to see what a step's ~700-800 cycles
// (per-wave stamps) are made of. Every lane of every wave walks its own ~300-byte
// text literal in an LDS window (all waves share the window and the image: their stores race, which
// changes nothing here), body steps only; cycles per step = s_memtime around the walk / the lane's
// steps, the wave's slowest lane. Variants:
//   0 the product body step (lit12_body<kPred, 3>: two lookups, four byte stores, LO branch)
//   1 the same without the stores (kNoStore)
//   2 the bare chain: window dword, two lookups, the bit position and the pair slide (no output)
//   3 two literals per lane stepped alternately (product step on each: two independent chains)
// at 1, 4 and 16 waves per CU (one workgroup). One JSON line per (variant, waves).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../loona_amd/csrc/hpk_wave.h"

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

using namespace hpkdec;

constexpr int kLitB = 304;                 // bytes per lane literal (window stride)
constexpr int kWinDw = 64 * 2 * kLitB / 4 + 16;  // two literals per lane
constexpr int kImgLane = 512;              // image bytes per lane (shared by the waves)

template <int kVar>
__global__ __launch_bounds__(1024) void probe(const uint32_t* __restrict__ lut3, const uint16_t* __restrict__ lo,
                                              const uint32_t* __restrict__ win, const uint32_t* __restrict__ nbits,
                                              unsigned long long* out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[HPK_LUT_SIZE];
    __shared__ __attribute__((aligned(16))) uint16_t s_lo[HPK_LO_SIZE];
    __shared__ __attribute__((aligned(16))) uint32_t s_win[kWinDw];
    __shared__ __attribute__((aligned(16))) uint8_t s_img[64 * kImgLane + 256];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t t = tid; t < HPK_LUT_SIZE; t += blockDim.x) s_lut[t] = lut3[t];
    for (uint32_t t = tid; t < HPK_LO_SIZE; t += blockDim.x) s_lo[t] = lo[t];
    for (uint32_t t = tid; t < (uint32_t)kWinDw; t += blockDim.x) s_win[t] = win[t];
    __syncthreads();
    auto make = [&](Lit12& L, uint32_t k) {
        L.X = (lane * 2u + k) * kLitB * 8u + 31u;
        L.Eb = L.X + nbits[lane * 2u + k];
        L.o = lane * kImgLane + k * (kImgLane / 2);
        L.o0 = L.o;
        L.st = HPK_OK;
        lit12_load(L, s_win);
    };
    Lit12 L, N;
    make(L, 0);
    make(N, 1);
    uint32_t steps = 0, sink = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (kVar == 3) {
        bool bl = L.Eb - L.X >= kBodyMin, bn = N.Eb - N.X >= kBodyMin;
        while (__any(bl | bn)) {
            if (bl) lit12_body<kPred, 3>(L, s_win, s_lut, s_lo, s_img, bl);
            if (bn) lit12_body<kPred, 3>(N, s_win, s_lut, s_lo, s_img, bn);
            steps += 1;
        }
    } else {
        bool body = L.Eb - L.X >= kBodyMin;
        while (__any(body)) {
            if (body) {
                if (kVar == 0) lit12_body<kPred, 3>(L, s_win, s_lut, s_lo, s_img, body);
                if (kVar == 1) lit12_body<kNoStore, 3>(L, s_win, s_lut, s_lo, s_img, body);
                if (kVar == 2) {
                    const uint32_t d3 = s_win[(L.X >> 5) + 2];
                    const uint32_t w = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
                    const uint32_t e1 = s_lut[w >> 20];
                    const uint32_t u1 = HPK_L3_HELD(e1);
                    const uint32_t e2 = s_lut[(w << u1) >> 20];
                    const uint32_t xn = L.X + u1 + HPK_L3_HELD(e2) + (HPK_L3_HELD(e2) == 0u ? 13u : 0u);
                    const bool cross = (xn ^ L.X) > 31u;
                    L.d0 = cross ? L.d1 : L.d0;
                    L.d1 = cross ? L.d2 : L.d1;
                    L.d2 = cross ? d3 : L.d2;
                    L.X = xn;
                    sink += e1 ^ e2;
                    body = L.Eb - L.X >= kBodyMin;
                }
            }
            steps += body ? 1u : 0u;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    // the wave's slowest lane: its steps
    uint32_t ms = steps;
    for (int d = 32; d >= 1; d >>= 1) ms = max(ms, (uint32_t)__shfl_xor((int)ms, d));
    if (lane == 0) {
        out[(tid >> 6) * 2] = t1 - t0;
        out[(tid >> 6) * 2 + 1] = ms + (sink == 0x12345u ? 1u : 0u) + (L.o == 0x7FFFFFFFu ? 1u : 0u);
    }
}

int main() {
    static hpk_tables T;
    if (hpk_build_tables(&T)) return 1;
    // text literals: letters, digits and punctuation (header-value like), 2 per lane
    const char* text = "abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:abcdefghijklmnopqrstuvwxyzeeeetttaaooiinnsshhrr";
    std::vector<uint8_t> winb(kWinDw * 4, 0);
    std::vector<uint32_t> nb(128);
    srand(7541);
    for (int l = 0; l < 128; ++l) {
        uint64_t acc = 0;
        int nacc = 0, pos = l * kLitB;
        const int end = pos + kLitB - 8;
        while (pos < end) {
            const uint8_t c = (uint8_t)text[rand() % 94];
            acc = (acc << T.len[c]) | T.code[c];
            nacc += T.len[c];
            while (nacc >= 8 && pos < end) {
                winb[pos++] = (uint8_t)(acc >> (nacc - 8));
                nacc -= 8;
            }
        }
        nb[l] = (uint32_t)(kLitB - 8) * 8u;
    }
    std::vector<uint32_t> w32(kWinDw);
    for (int i = 0; i < kWinDw; ++i)
        w32[i] = ((uint32_t)winb[4 * i] << 24) | ((uint32_t)winb[4 * i + 1] << 16) | ((uint32_t)winb[4 * i + 2] << 8) | winb[4 * i + 3];
    uint32_t *d_lut, *d_win, *d_nb;
    uint16_t* d_lo;
    unsigned long long* d_out;
    CK(hipMalloc(&d_lut, sizeof(T.lut3)));
    CK(hipMalloc(&d_lo, sizeof(T.lo)));
    CK(hipMalloc(&d_win, w32.size() * 4));
    CK(hipMalloc(&d_nb, nb.size() * 4));
    CK(hipMalloc(&d_out, 64 * 8));
    CK(hipMemcpy(d_lut, T.lut3, sizeof(T.lut3), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lo, T.lo, sizeof(T.lo), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_win, w32.data(), w32.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_nb, nb.data(), nb.size() * 4, hipMemcpyHostToDevice));
    auto run = [&](int var, int waves) {
        unsigned long long h[32];
        for (int rep = 0; rep < 3; ++rep) {
            switch (var) {
                case 0: hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64 * waves), 0, 0, d_lut, d_lo, d_win, d_nb, d_out); break;
                case 1: hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64 * waves), 0, 0, d_lut, d_lo, d_win, d_nb, d_out); break;
                case 2: hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64 * waves), 0, 0, d_lut, d_lo, d_win, d_nb, d_out); break;
                default: hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64 * waves), 0, 0, d_lut, d_lo, d_win, d_nb, d_out); break;
            }
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
        }
        CK(hipMemcpy(h, d_out, 2 * 8 * waves, hipMemcpyDeviceToHost));
        double cyc = 0, st = 0;
        for (int w = 0; w < waves; ++w) {
            cyc += (double)h[2 * w];
            st += (double)h[2 * w + 1];
        }
        printf("{\"variant\": %d, \"waves\": %d, \"cycles_per_wave\": %.0f, \"steps\": %.1f, \"cycles_per_step\": %.1f}\n",
               var, waves, cyc / waves, st / waves, cyc / st);
    };
    for (int var = 0; var < 4; ++var)
        for (int waves : {1, 4, 16}) run(var, waves);
    return 0;
}
