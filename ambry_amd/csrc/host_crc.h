// host_crc.h -- host (CPU) streaming CRC-32 behind ambrycrc_update.
//
// The register is the bit-inverted CRC, as Crc32.java keeps it (Crc32.java:37-52).
// host_update_reg dispatches once per process to the widest carry-less-multiply
// fold the CPU has (AVX-512 VPCLMULQDQ, then SSE PCLMULQDQ) and to slice-by-8
// (the reference's own loop, Crc32.java:55-98) for short inputs and CPUs without
// CLMUL. AMBRYCRC_HOST_IMPL=slice8|pclmul|vpclmul forces one (tests, benches).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace ambrycrc {

enum HostImpl { kHostSlice8 = 0, kHostPclmul = 1, kHostVpclmul = 2 };

uint32_t host_update_reg(uint32_t reg, const uint8_t* p, size_t n);
uint32_t host_update_slice8(uint32_t reg, const uint8_t* p, size_t n);
int host_impl();                   // the implementation host_update_reg uses
const char* host_impl_name(int impl);

}  // namespace ambrycrc
