/* gnsscorr_internal.h -- shared constants and internal helpers. */
#ifndef GNSSCORR_INTERNAL_H
#define GNSSCORR_INTERNAL_H
#include "gnsscorr.h"

/* Flat E/P/L image layout, as gcc places the reference's three statics
 * gps_prn_{early,prompt,late}[33][2046] (correlator.c:25-27): late first,
 * then prompt, then early, each followed by 2 pad bytes (nm -n of the
 * reference build).  Over-read indices >= 2046 walk into the next row. */
#define GNSSCORR_OSG_ROW_BYTES  2046
#define GNSSCORR_OSG_TAB        (GNSSCORR_OSG_ROW * 33)
#define GNSSCORR_OSG_OFF_LATE   0
#define GNSSCORR_OSG_OFF_PROMPT (GNSSCORR_OSG_TAB + 2)
#define GNSSCORR_OSG_OFF_EARLY  (2 * (GNSSCORR_OSG_TAB + 2))
/* packed-table entries: prn*2046 + uint16 index */
#define GNSSCORR_OSG_PK_LEN     (32 * GNSSCORR_OSG_ROW + 65536)
#define GNSSCORR_OSG_IMG_BYTES  (GNSSCORR_OSG_OFF_EARLY + GNSSCORR_OSG_PK_LEN + 256)

#ifdef __cplusplus
extern "C" {
#endif
void gnsscorr_osg_table_image(int8_t *img);
void gnsscorr_osg_packed_table(uint32_t *pk);
void gnsscorr_set_error(const char *fmt, ...);
int gnsscorr_track_iq(const gnsscorr_track_ctx *ctx);
/* GPS-SDR tables (sdr_host.c): packed (i, q) int16 pairs, N = 2048 */
void gnsscorr_sdr_twiddles(int16_t *w, int16_t *iw);
void gnsscorr_sdr_code_gen(int sv, uint8_t *chips);
void gnsscorr_sdr_post_dft(int16_t *out);
#ifdef __cplusplus
}
#endif
#endif
