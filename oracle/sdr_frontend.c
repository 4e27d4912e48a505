/* oracle/sdr_frontend.c -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).
 *
 * Scalar restatement of the GPS-SDR sample front end, loop for loop:
 *   GPS_Source::Read_GN3S     SDR/objects/gps_source.cpp:684-767 (5-ms branch)
 *   GPS_Source::Resample_GN3S SDR/objects/gps_source.cpp:933-943
 *   gdec table                SDR/objects/gps_source.cpp:433-437
 *   sin/cos tables, phase     SDR/objects/gps_source.cpp:92-96
 *   downsample                SDR/accessories/misc.cpp:174-197
 * The GPS_Source class does not build here (gn3s / usrp headers), so
 * Read_GN3S is restated; downsample is pinned to the reference build
 * (oracle/_ref/libsdr_ref.so, ref_sdr_downsample).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "sdr_frontend.h"

/* One 5-ms GN3S read: 20000 input bytes (low 2 bits used) -> 10240 CPX.
 * buff_tail: the reference's buff[20000], which Read_GN3S never writes. */
void orc_gn3s_block(const uint8_t *gbuff, uint32_t *phase, uint32_t delta, int16_t *out,
                    const int16_t *buff_tail)
{
  static const int16_t LUT[4] = {-3, -1, 1, 3};
  static double sin_table[1024], cos_table[1024];
  static int init = 0;
  static int16_t buff[40932][2];
  int lcv;
  if (!init) {
    for (int i = 0; i < 1024; i = i + 1) {
      sin_table[i] = -8 * sin(2 * M_PI * i / 1024);
      cos_table[i] = +8 * cos(2 * M_PI * i / 1024);
    }
    init = 1;
  }
  buff[20000][0] = buff_tail ? buff_tail[0] : 0;
  buff[20000][1] = buff_tail ? buff_tail[1] : 0;
  for (lcv = 0; lcv < 20000; lcv++) {
    const unsigned short_phase = *phase >> 22;
    buff[lcv][1] = (int16_t)(LUT[gbuff[lcv] & 0x03] * sin_table[short_phase]);
    buff[lcv][0] = (int16_t)(LUT[gbuff[lcv] & 0x03] * cos_table[short_phase]);
    *phase = *phase + delta;
  }
  for (int i = 0; i < 10240; i++) {
    const int g = (int)floor((i + 1) * 4000 / 2048);
    out[2 * i] = buff[g][0];
    out[2 * i + 1] = buff[g][1];
  }
}

int orc_downsample(int16_t *dest, const int16_t *source, double fdest, double fsource, int samps)
{
  int k = 0;
  uint32_t phase_step = (uint32_t)floor((double)4294967296.0 * fdest / fsource);
  uint32_t lphase = 0, phase = 0;
  for (int lcv = 0; lcv < samps; lcv++) {
    if (phase <= lphase) {
      dest[2 * k] = source[2 * lcv];
      dest[2 * k + 1] = source[2 * lcv + 1];
      k++;
    }
    lphase = phase;
    phase += phase_step;
  }
  return k;
}
