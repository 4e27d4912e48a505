/* tests/sanitize/san_driver.c -- TEST SCAFFOLDING: exercises the host C of the
 * library (csrc/codes.c, csrc/sdr_host.c, csrc/osg_legacy.c, csrc/common.c)
 * under -fsanitize=address,undefined (tests/test_sanitize_host.py).  Exit 0
 * and no sanitizer report = pass. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gnsscorr.h"
#include "gnsscorr_osg.h"
#include "gnsscorr_internal.h"

int main(void)
{
  int8_t code[1023], st[511];
  for (int prn = 1; prn <= 51; prn++)
    if (gnsscorr_ca_code(prn, code) != GNSSCORR_OK && prn <= 32) return 1;
  if (gnsscorr_ca_code(0, code) == GNSSCORR_OK || gnsscorr_ca_code(99, code) == GNSSCORR_OK) return 2;
  gnsscorr_st_code(st);
  int8_t *sc = malloc(16368);
  gnsscorr_ca_code(7, code);
  if (gnsscorr_sample_code(code, 1023, 1.023e6, 16.368e6, 16368, sc)) return 3;
  if (gnsscorr_sample_code(st, 511, 0.511e6, 16.0e6, 16000, sc)) return 4;
  free(sc);
  int8_t *img = malloc(GNSSCORR_OSG_IMG_BYTES);
  gnsscorr_osg_table_image(img);
  uint32_t *pk = malloc(sizeof(uint32_t) * GNSSCORR_OSG_PK_LEN);
  gnsscorr_osg_packed_table(pk);
  free(pk);
  free(img);
  gnsscorr_sig sigs[3];
  memset(sigs, 0, sizeof sigs);
  sigs[0].system = 0; sigs[0].prn = 5; sigs[0].code_phase = 100.25; sigs[0].doppler = 1200;
  sigs[0].cn0 = 48; sigs[0].data_bits = 1;
  sigs[1].system = 1; sigs[1].fch = -7; sigs[1].code_phase = 3; sigs[1].doppler = -900;
  sigs[1].cn0 = 45;
  sigs[2] = sigs[0]; sigs[2].prn = 32; sigs[2].code_phase = -5.5;
  const int64_t n = (1 << 20) + 77;   /* > 1 chunk: the threaded path */
  int8_t *iq = malloc(2 * n);
  if (gnsscorr_ifgen(iq, n, 1, 16.368e6, 2.42e6, 1.0e6, 3, sigs, 42)) return 5;
  if (gnsscorr_ifgen(iq, 1000, 0, 16.0e6, 2.42e6, 1.0e6, 3, sigs, 0)) return 6;
  /* GPS-SDR host tables */
  int16_t *tab = malloc(sizeof(int16_t) * 51 * 2048 * 2);
  if (gnsscorr_sdr_prn_codes(tab)) return 7;
  gnsscorr_sdr_sine_gen(tab, -38400.0 - 250.0, 2048000.0, 20480);
  gnsscorr_sdr_twiddles(tab, tab + 2048);
  gnsscorr_sdr_post_dft(tab);
  gnsscorr_sdr_gn3s_products(tab);
  uint8_t chips[1023];
  for (int sv = 0; sv < 51; sv++) gnsscorr_sdr_code_gen(sv, chips);
  free(tab);
  /* OSG register shim over the host stand-in of the tracking context */
  if (gnsscorr_osg_configure(16.368e6, 2.42e6, 0.0, 5.0, 30, 29, 12, 1, 1000.0, 0)) return 8;
  correlator_init(0.0);
  for (int ch = 0; ch < 12; ch++) {
    REG_write[ch << 3] = 1 + ch;
    REG_write[(ch << 3) + 3] = 9689; REG_write[(ch << 3) + 4] = 12345;
    REG_write[(ch << 3) + 5] = 102;  REG_write[(ch << 3) + 6] = 26214;
    REG_write[(ch << 3) + 7] = ch & 1 ? -1 : 3;
    REG_write[(ch << 3) + 0x84] = ch;
  }
  for (int call = 0; call < 10; call++) Sim_GP2021_int((char *)iq + call * 2 * 8380, 8380);
  correlator_init(0.0);              /* re-init keeps the ms/bit counters */
  Sim_GP2021_int((char *)iq, 8380);
  free(iq);
  printf("sanitized host run OK (dump mask %x)\n", REG_read[0x82]);
  return 0;
}
