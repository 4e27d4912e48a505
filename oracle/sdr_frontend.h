/* oracle/sdr_frontend.h -- TEST INFRASTRUCTURE ONLY (see sdr_frontend.c). */
#ifndef ORACLE_SDR_FRONTEND_H
#define ORACLE_SDR_FRONTEND_H
#include <stdint.h>
void orc_gn3s_block(const uint8_t *gbuff, uint32_t *phase, uint32_t delta, int16_t *out,
                    const int16_t *buff_tail);
int orc_downsample(int16_t *dest, const int16_t *source, double fdest, double fsource, int samps);
#endif
