// lds_tr.h -- MFMA operand fragments read TRANSPOSED from LDS with the gfx950 ds_read_b64_tr_b8.
//
// Probed on MI355X (scratch/probe/tr8.hip): in each 16-lane group, lane j supplies the LDS address
// of 8 bytes C[j]; lane i then receives byte (i & 7) of C[2k + (i >> 3)] as its byte k, k = 0..7 --
// i.e. lanes 2r, 2r+1 form row r (16 bytes) of an 8 x 16 block and lane i gets column i.
// So for an image of [pixel][16 channel bytes] rows, two reads deliver, in lane l of group g,
// channel (l & 15) of the 16 consecutive pixels 16g' .. 16g'+15 -- the A[row][k] / B[k][col]
// fragment of v_mfma_i32_16x16x64_i8 with k = pixels (the weight-gradient GEMMs).
#pragma once
#include "dfxp_device.h"

namespace lbt {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

// 16 pixels (rows base..base+15 of a [pixel][16 B] image) of channel (lane & 15): 16 bytes
LBT_DEV v4i tr_frag(const int8_t* img, int base, int lane) {
  const int j = lane & 15;
  const int8_t* p0 = img + (base + (j >> 1)) * 16 + 8 * (j & 1);
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(p0));
  const v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(p0 + 8 * 16));
  return v4i{lo.x, lo.y, hi.x, hi.y};
}

}  // namespace lbt
