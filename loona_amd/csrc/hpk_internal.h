// hpk_internal.h — declarations shared between the host (hpk_cpu.cpp) and device (hpk_gpu.hip)
// halves of libhpk. Not part of the C ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "hpk_code.h"

const hpk_tables* hpk_get_tables();
int hpk_cpu_decode(const hpk_tables* t, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                   size_t* out_len);
int hpk_cpu_encode(const hpk_tables* t, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                   size_t* out_len);
