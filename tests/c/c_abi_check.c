/* c_abi_check.c -- include/lbf_hash.h consumed from plain C99 (test input of
 * tests/test_abi.py::test_header_is_plain_c).  No hashing happens unless a GPU
 * is visible: on a CPU-only host the context must refuse with
 * LBF_ERR_NO_DEVICE, and the host-side base64-27 helpers must still work. */
#include <stdio.h>
#include <string.h>

#include "lbf_hash.h"

int main(void) {
  /* SHA-1("abc"), Crypto++ TestVectors/sha.txt */
  static const uint8_t abc[20] = {0xa9, 0x99, 0x3e, 0x36, 0x47, 0x06, 0x81, 0x6a, 0xba, 0x3e,
                                  0x25, 0x71, 0x78, 0x50, 0xc2, 0x6c, 0x9c, 0xd0, 0xd8, 0x9d};
  char s[LBF_B64_CHARS + 1];
  uint8_t back[LBF_DIGEST_BYTES];
  lbf_ctx* ctx = NULL;
  int ndev = -1, rc;
  if (lbf_abi_version() != LBF_ABI_VERSION) return 10;
  lbf_b64_27(abc, s);
  if (strcmp(s, "qZk+NkcGgWq6PiVxeFDCbJzQ2J0") != 0) return 11;
  if (lbf_b64_27_decode(s, strlen(s), back) != LBF_OK || memcmp(back, abc, 20) != 0) return 12;
  if (lbf_device_count(&ndev) != LBF_OK) return 13;
  rc = lbf_ctx_create(0, &ctx);
  if (ndev == 0) {
    if (rc != LBF_ERR_NO_DEVICE || ctx != NULL) return 14;
    printf("ok: no device, ctx refused: %s\n", lbf_last_error());
    return 0;
  }
  if (rc != LBF_OK) return 15;
  {
    uint8_t d[20];
    if (lbf_sha1_one(ctx, (const uint8_t*)"abc", 3, d) != LBF_OK || memcmp(d, abc, 20) != 0) return 16;
  }
  lbf_ctx_destroy(ctx);
  printf("ok: %d device(s), SHA-1(abc) on the GPU matches\n", ndev);
  return 0;
}
