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
/* n_calls closed-loop calls in ONE launch (track.hip osg_stream_kernel): each
 * channel's wave correlates call k, runs its gpsisr step and goes on to call
 * k+1 with the new command words; d_res / d_loop_hist receive every call.
 * GNSSCORR_TRACK_NOT_FUSED when that kernel does not serve the context (I-only
 * streams, A/B switches, shapes) or n_loops differs from the context's channel
 * count; the caller then runs the calls as correlator + osg_isr_kernel launches. */
#define GNSSCORR_TRACK_NOT_FUSED 1
int gnsscorr_track_dev_isr(gnsscorr_track_ctx *ctx, const int8_t *d_if, int64_t stream_stride,
                           int64_t nsamp, int n_calls, gnsscorr_nco_cmd *d_cmds,
                           gnsscorr_track_result *d_res, int n_loops,
                           const gnsscorr_osg_loop_cfg *cfg, gnsscorr_osg_loop *d_loops,
                           gnsscorr_osg_loop *d_loop_hist);
/* GPS-SDR tables (sdr_host.c): packed (i, q) int16 pairs, N = 2048 */
void gnsscorr_sdr_twiddles(int16_t *w, int16_t *iw);
void gnsscorr_sdr_code_gen(int sv, uint8_t *chips);
void gnsscorr_sdr_post_dft(int16_t *out);
#ifdef __cplusplus
}
#endif
#endif
