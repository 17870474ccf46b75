// kvariants.hip — development harness (not part of the product): times decode-kernel variants
// (refill period, ILP) on one batch in a single process and checks each against the library's
// CPU path (hpk_decode_batch_cpu, itself pinned to the oracle by tests/test_host.py).
// Input file (written by scripts/kinput.py): u32 n, u32 enc_bytes, u32 in_off[n+1], u8 blob[].
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "legacy_decode11.h"
#include "legacy_decode12.h"

using namespace hpkdec;

int hpk_set_err(const char*, hipError_t) { return -3; }
int hpk_set_err_msg(const char*, int c) { return c; }

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                               \
        }                                                                          \
    } while (0)

struct Dev {
    DecodeArgs a;
    uint32_t n;
    size_t out_bytes;
};

template <int kMode, class Fn>
static void run_fn(const char* name, Fn fn, int lds, int block, int blocks_per_cu, Dev& d,
                   const std::vector<uint32_t>& ref_len, const std::vector<uint8_t>& ref_st,
                   const std::vector<uint8_t>& ref_out, int num_cu, int iters) {
    if (lds) CK(hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    dim3 grid(num_cu * blocks_per_cu), blk(block);
    CK(hipMemset(d.a.out_len, 0xFF, d.n * 4));
    CK(hipMemset(d.a.out_base, 0xAB, d.out_bytes));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(fn, grid, blk, lds, 0, d.a);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(fn, grid, blk, lds, 0, d.a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint32_t> len(d.n);
    std::vector<uint8_t> st(d.n), out(d.out_bytes);
    CK(hipMemcpy(len.data(), d.a.out_len, d.n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(st.data(), d.a.status, d.n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(out.data(), d.a.out_base, d.out_bytes, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint32_t i = 0; i < d.n; ++i)
        if (len[i] != ref_len[i] || st[i] != ref_st[i]) ++bad;
    std::vector<uint32_t> oo(d.n + 1);
    CK(hipMemcpy(oo.data(), d.a.out_off, (d.n + 1) * 4, hipMemcpyDeviceToHost));
    size_t badb = 0;
    if (kMode == 0 || kMode == 4)
        for (uint32_t i = 0; i < d.n; ++i)
            if (memcmp(&out[oo[i]], &ref_out[oo[i]], ref_len[i]) != 0) ++badb;
    unsigned long long chk[8] = {0};
    if (kMode == 4) CK(hipMemcpyFromSymbol(chk, HIP_SYMBOL(g_chk), sizeof chk));
    printf("{\"variant\": \"%s\", \"us\": %.2f, \"bad_len_status\": %zu, \"bad_bytes\": %zu, \"chk\": [%llu, %llu, %llu, %llu]}\n",
           name, ms * 1000.0 / iters, bad, badb, chk[0], chk[1], chk[2], chk[3]);
    fflush(stdout);
}

// v5: block window + block queue, output stored straight to global
template <int kMode, int kW, int kD, int kM, int kR, int kC, int kBlocksPerCu = 1, int kStep = 4>
static void run(const char* name, Dev& d, const std::vector<uint32_t>& ref_len, const std::vector<uint8_t>& ref_st,
                const std::vector<uint8_t>& ref_out, int num_cu, int iters) {
    using G = BlockGeometry<kW, kD, kM>;
    run_fn<kMode>(name, hpk_decode_kernel<kMode, kW, kD, kM, kR, kC, kStep>, G::kLdsBytes, G::kBlock, kBlocksPerCu, d,
                  ref_len, ref_st, ref_out, num_cu, iters);
}

// v7: input window + output image in LDS, longest-first queue
template <int kMode, int kWaves, int kW, int kO, int kQ, int kR, int kC, int kStep, int kBlocksPerCu = 1>
static void run7(const char* name, Dev& d, const std::vector<uint32_t>& ref_len, const std::vector<uint8_t>& ref_st,
                 const std::vector<uint8_t>& ref_out, int num_cu, int iters) {
    using G = Geo7<kWaves, kW, kO, kQ, (kStep >= 8)>;
    run_fn<kMode>(name, hpk_decode7<kMode, kWaves, kW, kO, kQ, kR, kC, kStep>, 0, G::kBlock, kBlocksPerCu,
                  d, ref_len, ref_st, ref_out, num_cu, iters);
}

// v11: one big window per fill, output dwords straight to global
template <int kMode, int kWaves, int kW, int kQ, int kR, int kC, bool kLpt = true>
static void run11(const char* name, Dev& d, const std::vector<uint32_t>& ref_len, const std::vector<uint8_t>& ref_st,
                  const std::vector<uint8_t>& ref_out, int num_cu, int iters) {
    using G = Geo11<kWaves, kW, kQ>;
    run_fn<kMode>(name, hpk_decode11<kMode, kWaves, kW, kQ, kR, kC, kLpt>, 0, G::kBlock, 1, d, ref_len, ref_st, ref_out,
                  num_cu, iters);
}

// v12: bit-position step (kLook lookups per step, byte or dword stores) + cooperative long literals
static const char* g_only = nullptr;  // run only the variant of this name (argv[3])

template <int kMode, int kR, int kLook, bool kAcc, int kWaves = 16, int kW = 40960, int kO = 79104, int kQ = 2048,
          int kCoop = 1, int kBlocksPerCu = 1, int kSched = 0, int kLongDyn = 1, int kDefer = 0, int kPredSt = 1,
          int kSpread = 0, int kSmallFill = 512, uint32_t kLead = 0, int kEven = 1, int kSegBig = 15, int kSegSmall = 32>
static void run12(const char* name, Dev& d, const std::vector<uint32_t>& ref_len, const std::vector<uint8_t>& ref_st,
                  const std::vector<uint8_t>& ref_out, int num_cu, int iters) {
    if (g_only && strcmp(g_only, name) != 0) return;
    using G = Geo12<kWaves, kW, kO, kQ>;
    run_fn<kMode>(name, hpk_decode12<kMode, kWaves, kW, kO, kQ, kR, 64, kLook, kAcc, kCoop, kSched, kLongDyn, kDefer, kPredSt, kSpread, kSmallFill, kLead, kEven, kSegBig, kSegSmall>, 0, G::kBlock, kBlocksPerCu,
                  d, ref_len, ref_st, ref_out, num_cu, iters);
}

// v12 diagnostic stamps (kMode 3): per wave total cycles, cycles in the decode phases, steps, fills
template <int kR, int kLook, bool kAcc, int kWaves = 16, int kW = 40960, int kO = 79104, int kQ = 2048, int kSched = 0,
          int kLongDyn = 1, int kDefer = 0, int kPredSt = 1, int kSpread = 0, int kSmallFill = 512, uint32_t kLead = 0,
          int kEven = 1, int kCoop = 1>
static void stamps12(const char* name, Dev& d, int num_cu) {
    using G = Geo12<kWaves, kW, kO, kQ>;
    const size_t nw = (size_t)num_cu * kWaves;
    unsigned long long* dbg;
    CK(hipMalloc(&dbg, nw * 16 * 8));
    DecodeArgs a = d.a;
    a.dbg = dbg;
    auto fn = hpk_decode12<3, kWaves, kW, kO, kQ, kR, 64, kLook, kAcc, kCoop, kSched, kLongDyn, kDefer, kPredSt, kSpread, kSmallFill, kLead, kEven>;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(fn, dim3(num_cu), dim3(G::kBlock), 0, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(nw * 16);
    CK(hipMemcpy(h.data(), dbg, nw * 128, hipMemcpyDeviceToHost));
    double s[14] = {0}, mx[14] = {0};
    for (size_t w = 0; w < nw; ++w)
        for (int j = 0; j < 14; ++j) {
            s[j] += (double)h[w * 16 + j];
            mx[j] = std::max(mx[j], (double)h[w * 16 + j]);
        }
    printf("{\"stamps\": \"%s\", \"cycles_mean\": %.0f, \"cycles_max\": %.0f, \"decode_cycles_mean\": %.0f, "
           "\"decode_cycles_max\": %.0f, \"steps_mean\": %.1f, \"steps_max\": %.0f, \"barrier_wait_mean\": %.0f, "
           "\"pre_mean\": %.0f, \"setupA_mean\": %.0f, \"setupB_mean\": %.0f, \"long_mean\": %.0f, \"long_max\": %.0f, "
           "\"setupA_fill0\": %.0f, \"setupB_fill0\": %.0f, \"byte_pass\": %.0f, \"last_flush\": %.0f, "
           "\"long_literals\": %.0f, \"resync_rounds_per_long\": %.2f}\n",
           name, s[0] / nw, mx[0], s[1] / nw, mx[1], s[2] / nw, mx[2], s[3] / nw, s[4] / nw, s[5] / nw, s[6] / nw,
           s[7] / nw, mx[7], s[8] / nw, s[9] / nw, s[10] / nw, s[11] / nw, s[13],
           s[13] > 0 ? s[12] / s[13] : 0.0);
    fflush(stdout);
    CK(hipFree(dbg));
}

extern "C" int hpk_decode_batch_cpu(const uint8_t*, const uint32_t*, uint32_t, uint8_t*, const uint32_t*, uint32_t*,
                                    uint8_t*, int);

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    setvbuf(stdout, nullptr, _IOLBF, 0);
    FILE* f = fopen(argv[1], "rb");
    uint32_t n, eb;
    if (fread(&n, 4, 1, f) != 1 || fread(&eb, 4, 1, f) != 1) return 1;
    std::vector<uint32_t> in_off(n + 1);
    std::vector<uint8_t> blob(eb + 16);
    if (fread(in_off.data(), 4, n + 1, f) != n + 1 || fread(blob.data(), 1, eb, f) != eb) return 1;
    fclose(f);
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    std::vector<uint32_t> out_off(n + 1);
    out_off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) out_off[i + 1] = out_off[i] + ((((in_off[i + 1] - in_off[i]) * 8) / 5 + 3) & ~3u);
    const size_t ob = out_off[n] + 16;
    std::vector<uint8_t> ref_out(ob);
    std::vector<uint32_t> ref_len(n);
    std::vector<uint8_t> ref_st(n);
    hpk_decode_batch_cpu(blob.data(), in_off.data(), n, ref_out.data(), out_off.data(), ref_len.data(), ref_st.data(), 0);

    hpk_tables tab;
    hpk_build_tables(&tab);
    Dev d;
    d.n = n;
    d.out_bytes = ob;
    uint8_t *d_in, *d_out, *d_st;
    uint32_t *d_io, *d_oo, *d_len, *d_lut, *d_lut2;
    uint16_t* d_lo;
    CK(hipMalloc(&d_in, eb + 64));
    CK(hipMalloc(&d_out, ob));
    CK(hipMalloc(&d_st, n));
    CK(hipMalloc(&d_io, (n + 1) * 4));
    CK(hipMalloc(&d_oo, (n + 1) * 4));
    CK(hipMalloc(&d_len, n * 4));
    CK(hipMalloc(&d_lut, sizeof(tab.t8)));
    CK(hipMalloc(&d_lo, sizeof(tab.lo)));
    CK(hipMalloc(&d_lut2, sizeof(tab.lut)));
    CK(hipMemcpy(d_lut2, tab.lut, sizeof(tab.lut), hipMemcpyHostToDevice));
    uint32_t* d_lut3;
    CK(hipMalloc(&d_lut3, sizeof(tab.lut2)));
    CK(hipMemcpy(d_lut3, tab.lut2, sizeof(tab.lut2), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_in, blob.data(), eb, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_io, in_off.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_oo, out_off.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lut, tab.t8, sizeof(tab.t8), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lo, tab.lo, sizeof(tab.lo), hipMemcpyHostToDevice));
    DecodeArgs& a = d.a;
    a.in_base = d_in;
    a.in_mis = 0;
    a.in_off = d_io;
    a.n = n;
    a.out_base = d_out;
    a.out_mis = 0;
    a.out_off = d_oo;
    a.out_len = d_len;
    a.status = d_st;
    a.t8 = reinterpret_cast<const uint8_t*>(d_lut);
    a.lo = d_lo;
    a.lut = d_lut2;
    a.lut2 = d_lut3;
    a.dbg = nullptr;
    a.in_cap = eb;
    a.out_cap = (uint32_t)ob;
    uint32_t* d_err;
    CK(hipMalloc(&d_err, 4));
    CK(hipMemset(d_err, 0, 4));
    a.err = d_err;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cu = prop.multiProcessorCount;
    printf("{\"n\": %u, \"enc_bytes\": %u, \"cus\": %d}\n", n, eb, cu);
    if (argc > 3) {  // one named variant per process (a hang then names itself)
        g_only = argv[3];
        run12<0, 3, 2, false, 16, 40960, 79104, 2048, 0>("coop0", d, ref_len, ref_st, ref_out, cu, iters);
        run12<4, 3, 2, false>("coop1_checked", d, ref_len, ref_st, ref_out, cu, 1);
        run12<0, 3, 2, false>("coop1", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1>("coop1_snake", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 0>("snake_longstatic", d, ref_len, ref_st, ref_out, cu,
                                                                   iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 1>("snake_defer", d, ref_len, ref_st, ref_out, cu,
                                                                      iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 0>("snake_nopred", d, ref_len, ref_st, ref_out, cu,
                                                                         iters);
        run12<0, 2, 2, true, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1>("snake_acc_pred", d, ref_len, ref_st, ref_out, cu,
                                                                        iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 1>("snake_spread", d, ref_len, ref_st, ref_out, cu,
                                                                            iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 1, 0>("snake_spread_nosmall", d, ref_len, ref_st,
                                                                               ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 0, 0>("snake_nosmall", d, ref_len, ref_st, ref_out,
                                                                               cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 0, 512, 0>("snake_nolead", d, ref_len, ref_st,
                                                                                   ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 0, 512, 0, 0>("greedy", d, ref_len, ref_st, ref_out,
                                                                                      cu, iters);
        run12<0, 2, 2, false, 16, 36864, 83200, 2048, 1, 1, 1, 1, 0, 1, 0, 512, 0, 0>("w36_greedy", d, ref_len, ref_st,
                                                                                      ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 43008, 77056, 2048, 1, 1, 1>("w42", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 3, 2, false, 16, 40960, 79104, 2048, 1, 1, 1>("r3", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 1, 2, false, 16, 40960, 79104, 2048, 1, 1, 1>("r1", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 4, 2, false, 16, 40960, 79104, 2048, 1, 1, 1>("r4", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 45056, 75008, 2048, 1, 1, 1>("w44", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 38912, 81152, 2048, 1, 1, 1>("w38", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 36864, 83200, 2048, 1, 1, 1>("w36", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 34816, 85248, 2048, 1, 1, 1>("w34", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 32768, 87296, 2048, 1, 1, 1>("w32", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 28672, 91392, 2048, 1, 1, 1>("w28", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 0, 512, 24>("snake_lead24", d, ref_len, ref_st,
                                                                                    ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1, 0, 512, 96>("snake_lead96", d, ref_len, ref_st,
                                                                                    ref_out, cu, iters);
        run12<0, 3, 2, true, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1>("snake_acc_pred_r3", d, ref_len, ref_st, ref_out,
                                                                           cu, iters);
        run12<4, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1, 1, 0, 1>("snake_pred_checked", d, ref_len, ref_st, ref_out,
                                                                         cu, 1);
        // v18 segment stream: thresholds (buckets) big / small fill: 15 = 224 B, 32 = 64 B, 40 = 48 B, 48 = 32 B
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 3, 1, 1, 1, 0, 1, 0, 512, 0, 1, 15, 32>("seg_224_64", d, ref_len, ref_st, ref_out, cu, iters);
        run12<4, 2, 2, false, 16, 40960, 79104, 2048, 3, 1, 1, 1, 0, 1, 0, 512, 0, 1, 15, 32>("seg_224_64_checked", d, ref_len, ref_st, ref_out, cu, 1);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 3, 1, 1, 1, 0, 1, 0, 512, 0, 1, 15, 48>("seg_224_32", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 3, 1, 1, 1, 0, 1, 0, 512, 0, 1, 32, 48>("seg_64_32", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 16, 40960, 79104, 2048, 3, 1, 1, 1, 0, 1, 0, 512, 0, 1, 24, 40>("seg_128_48", d, ref_len, ref_st, ref_out, cu, iters);
        // two 512-thread workgroups per CU (<= 80 KiB of LDS each): one workgroup's fill setup,
        // barrier wait and write-back overlap the other's decode
        run12<0, 2, 2, false, 8, 18432, 32096, 1024, 1, 2, 1>("wg2_w18", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 8, 16384, 34144, 1024, 1, 2, 1>("wg2_w16", d, ref_len, ref_st, ref_out, cu, iters);
        run12<0, 2, 2, false, 8, 14336, 29696, 1024, 1, 2, 1>("wg2_w14", d, ref_len, ref_st, ref_out, cu, iters);
        run12<4, 2, 2, false, 8, 18432, 32096, 1024, 1, 2, 1>("wg2_w18_checked", d, ref_len, ref_st, ref_out, cu, 1);
        // three 256-thread workgroups per CU
        run12<0, 2, 2, false, 4, 10240, 17408, 512, 1, 3, 1>("wg3_w10", d, ref_len, ref_st, ref_out, cu, iters);
        if (!strcmp(g_only, "stamps")) {
            stamps12<2, 2, false, 16, 40960, 79104, 2048, 1>("coop1_snake", d, cu);
            stamps12<2, 2, false, 16, 40960, 79104, 2048, 1, 1, 0, 1, 0, 512, 0>("snake_nolead", d, cu);
            stamps12<2, 2, false, 16, 40960, 79104, 2048, 1, 0>("snake_longstatic", d, cu);
            stamps12<2, 2, false, 16, 40960, 79104, 2048, 1, 1, 0, 1, 0, 512, 0, 1, 3>("seg_224_64", d, cu);
        }
        return 0;
    }
    run12<0, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1>("v13_snake_r2", d, ref_len, ref_st, ref_out, cu, iters);
    run12<0, 2, 2, true, 16, 40960, 79104, 2048, 1, 1, 1>("v13_snake_acc_r2", d, ref_len, ref_st, ref_out, cu, iters);
    run12<2, 2, 2, false, 16, 40960, 79104, 2048, 1, 1, 1>("v13_snake_r2_nostore", d, ref_len, ref_st, ref_out, cu, iters);
    return 0;
}
