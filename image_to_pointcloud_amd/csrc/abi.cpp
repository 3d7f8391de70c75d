// ABI bookkeeping: version and thread-local last-error string.
#include "common.h"

#include <cstring>

namespace i2pc {

static thread_local char g_err[512] = {0};

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { g_err[0] = 0; }

}  // namespace i2pc

extern "C" int i2pc_abi_version(void) { return 1; }

extern "C" const char* i2pc_last_error(void) { return i2pc::g_err; }

bool i2pc_gemm_tune(const char* name, int value);        // gemm.hip
bool i2pc_unproject_tune(const char* name, int value);   // unproject.hip
bool i2pc_attention_tune(const char* name, int value);   // attention.hip
bool i2pc_misc_tune(const char* name, int value);        // misc.hip

extern "C" int i2pc_set_tuning(const char* name, int value) {
  i2pc::clear_error();
  I2PC_REQUIRE(name, "NULL tuning name");
  if (i2pc_gemm_tune(name, value) || i2pc_unproject_tune(name, value) || i2pc_attention_tune(name, value) ||
      i2pc_misc_tune(name, value))
    return I2PC_OK;
  return i2pc::set_error(I2PC_EINVAL,
                         "unknown tuning knob '%s' (gemm_tail, gemm_bn128, gemm_splitk, gemm_split_tile, gemm_tile192, gemm_lnp_p, gemm_lnp_stream, conv_halo, gelu_tanh, gemm_resq, gemm_simple_epi, gemm_tail160, gemm_stagger, "
                         "unp_rows, unp_nt, unp_rpt, sel_windows, sel_parts, sel_rows, sel_lband, sel_scratch, attn_lazy, attn_scalar, attn_rb, "
                         "ln_f2, ln_apply_gs, resize_rows: include/i2pc.h)",
                         name);
}
