// Host AddressSanitizer run of the C ABI's argument checks (SURVEY.md §5 "Race detection /
// sanitizers").  Built by tests/asan/build.sh with the library source compiled
// host-only under -fsanitize=address (no device code: every call below must be refused before any
// kernel launch), then run by tests/test_abi_asan.py.  Prints one line per check; exit 0 = all held.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "cnmf_hip.h"

static int g_fail = 0;
#define EXPECT(cond, what)                                                              \
  do {                                                                                  \
    if (!(cond)) {                                                                      \
      std::printf("FAIL %s (last error: %s)\n", what, cnmf_last_error());                \
      ++g_fail;                                                                         \
    } else {                                                                            \
      std::printf("ok   %s\n", what);                                                   \
    }                                                                                   \
  } while (0)

int main() {
  EXPECT(cnmf_abi_version() >= 300, "abi version");
  EXPECT(cnmf_padded_k(0) < 0 && cnmf_padded_k(17) < 0 && cnmf_padded_k(5) == 8, "padded k");
  EXPECT(cnmf_stage_doubles(340) == 64 * 340, "stage doubles");
  EXPECT(cnmf_mu_sample_pass(nullptr, 0, nullptr, nullptr, nullptr, nullptr, 10, 81, 4, 0, 0, 3, nullptr) ==
             CNMF_ERR_ARG, "sample pass: null pointers");
  EXPECT(std::strstr(cnmf_last_error(), "null") != nullptr, "message names the null pointer");
  EXPECT(cnmf_pass_blocks(100, 81, 17, 0) == CNMF_ERR_UNSUPPORTED, "k > 16");
  EXPECT(cnmf_pass_blocks(100, 81, 4, 9) == CNMF_ERR_ARG, "unknown dtype");
  EXPECT(cnmf_pass_blocks(100, 0, 4, 0) == CNMF_ERR_SHAPE, "F < 1");
  char buf[16];
  EXPECT(cnmf_persist_describe(1024, 81, 4, 0, 7, buf, sizeof(buf)) == CNMF_ERR_ARG, "bad layout");
  EXPECT(cnmf_persist_describe(1024, 81, 4, 0, 0, nullptr, 16) == CNMF_ERR_ARG, "describe: null buffer");
  EXPECT(cnmf_mu_iterations(5, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 1, nullptr, nullptr,
                            nullptr, nullptr, 1024, 81, 4, 0, 0, 0, 0, -1, nullptr, 0, nullptr) == CNMF_ERR_ARG,
         "iterations: bad layout first");
  EXPECT(cnmf_mu_iterations(0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 1, nullptr, nullptr,
                            nullptr, nullptr, 1024, 81, 4, 0, 0, 0, 0, 0, nullptr, 0, nullptr) == CNMF_OK,
         "iterations: n_iter 0 is a no-op");
  EXPECT(cnmf_basis_update(nullptr, nullptr, nullptr, nullptr, 81, 4, 0, 0, 1, nullptr, nullptr) == CNMF_ERR_ARG,
         "basis update: null pointers");
  EXPECT(cnmf_xctl_words(0) == CNMF_ERR_ARG && cnmf_xctl_words(65) == CNMF_ERR_ARG, "xctl world range");
  EXPECT(cnmf_xctl_init(nullptr, nullptr, 0, 1) == CNMF_ERR_ARG, "xctl init: null");
  uint64_t xctl[16];
  void* peers[2] = {nullptr, nullptr};
  EXPECT(cnmf_xctl_init(xctl, peers, 2, 2) == CNMF_ERR_ARG, "xctl init: rank out of range");
  EXPECT(cnmf_xctl_init(xctl, peers, 0, 2) == CNMF_ERR_ARG, "xctl init: null peer buffer");
  EXPECT(cnmf_xbuf_bytes(0) == CNMF_ERR_ARG, "xbuf world 0");
  EXPECT(cnmf_xbuf_alloc(2, nullptr, nullptr) == CNMF_ERR_ARG, "xbuf alloc: null");
  EXPECT(cnmf_device_pci_bus_id(0, buf, 4) == CNMF_ERR_ARG, "pci bus id: buffer too small");
  EXPECT(cnmf_wmu_pass_blocks(10, 600, 4) == CNMF_ERR_UNSUPPORTED, "weighted: F > 512");
  EXPECT(cnmf_wmu_basis_update(nullptr, nullptr, 81, 4, nullptr) == CNMF_ERR_ARG, "weighted basis: null");
  EXPECT(cnmf_init_gram(nullptr, 0, 10, 81, nullptr, 1, nullptr) == CNMF_ERR_ARG, "init gram: null");
  EXPECT(cnmf_init_fill(nullptr, 10, 4, nullptr, nullptr, nullptr, 0, 0, nullptr, 0, nullptr) == CNMF_ERR_ARG,
         "init fill: null");
  EXPECT(cnmf_host_register(nullptr, 10) == CNMF_ERR_ARG, "host register: null");
  EXPECT(cnmf_copy_h2d_async(nullptr, nullptr, 8, nullptr) == CNMF_ERR_ARG, "h2d copy: null");
  EXPECT(cnmf_als_iterations_multi(3, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1,
                                   nullptr, nullptr, nullptr, 1024, 81, 4, 1, 0.5, nullptr, nullptr, 0, nullptr) ==
             CNMF_ERR_ARG, "ALS multi: null control block");
  // a long message through the thread-local buffer (vsnprintf bound)
  char big[2048];
  std::memset(big, 'x', sizeof(big) - 1);
  big[sizeof(big) - 1] = 0;
  EXPECT(cnmf_wmu_pass_blocks(-1, 81, 4) < 0 && std::strlen(cnmf_last_error()) < 512, "bounded message");
  std::printf("%d failure(s)\n", g_fail);
  return g_fail == 0 ? 0 : 1;
}
