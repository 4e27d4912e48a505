// oracle/sdr_chan_ref.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Drives the reference GPS-SDR Channel class itself (objects/channel.cpp,
// compiled from its own sources with -DNO_SIMD together with
// objects/threaded_object.cpp, objects/fft.cpp and simd/x86.cpp; recipe in
// oracle/Makefile, output only in oracle/_ref/).  Channel::Accum
// (channel.cpp:182-279) is called exactly as Correlator::DumpAccum calls it;
// the subframes ProcessDataBit writes to the CHN_2_EPH_P pipe (:687) are read
// back from a real pipe.  The receiver's globals come from the reference's own
// includes/globals.h (GLOBALS_HERE, as main/main.cpp does).  State is read
// through Telemetry, which channel.h:51 declares a friend of Channel.
#define GLOBALS_HERE
#include "includes.h"
#include "channel.h"
#include <fcntl.h>
#include <unistd.h>

// field order of gnsscorr_sdr_channel (include/gnsscorr.h)
struct RefChanState {
  double carrier_nco, code_nco;
  int32 len, count, state, sv, chan;
  int32 I[3], Q[3], P[3], I_prev, Q_prev;
  float I_avg, Q_var, P_avg, cn0;
  int32 bit_lock, bit_lock_pend, bit_lock_ticks, I_sum20, Q_sum20;
  int32 I_buff[20], Q_buff[20], P_buff[20];
  int32 _20ms_epoch, _1ms_epoch, best_epoch;
  int32 valid_frame[5], navigate, z_lock, converged, frame_z, z_count, z_count_pend;
  uint32 word_buff[FRAME_SIZE_PLUS_2];
  int32 frame_lock, frame_lock_pend, bit_number, subframe;
  int32 freq_lock, freq_lock_ticks;
  float pll[17];   // Phase_lock_loop floats: PLLBW .. t (fll_lock reads an uninitialised local)
  float dll[7];    // Delay_lock_loop
};

class Telemetry {
 public:
  static void get(Channel* c, RefChanState* s) {
    memset(s, 0, sizeof *s);
    s->carrier_nco = c->carrier_nco;
    s->code_nco = c->code_nco;
    s->len = c->len; s->count = c->count; s->state = c->state; s->sv = c->sv; s->chan = c->chan;
    for (int k = 0; k < 3; k++) { s->I[k] = c->I[k]; s->Q[k] = c->Q[k]; s->P[k] = c->P[k]; }
    s->I_prev = c->I_prev; s->Q_prev = c->Q_prev;
    s->I_avg = c->I_avg; s->Q_var = c->Q_var; s->P_avg = c->P_avg; s->cn0 = c->cn0;
    s->bit_lock = c->bit_lock; s->bit_lock_pend = c->bit_lock_pend;
    s->bit_lock_ticks = c->bit_lock_ticks; s->I_sum20 = c->I_sum20; s->Q_sum20 = c->Q_sum20;
    for (int k = 0; k < 20; k++) {
      s->I_buff[k] = c->I_buff[k]; s->Q_buff[k] = c->Q_buff[k]; s->P_buff[k] = c->P_buff[k];
    }
    s->_20ms_epoch = c->_20ms_epoch; s->_1ms_epoch = c->_1ms_epoch; s->best_epoch = c->best_epoch;
    for (int k = 0; k < 5; k++) s->valid_frame[k] = c->valid_frame[k];
    s->navigate = c->navigate; s->z_lock = c->z_lock; s->converged = c->converged;
    s->frame_z = c->frame_z; s->z_count = c->z_count; s->z_count_pend = c->z_count_pend;
    for (int k = 0; k < FRAME_SIZE_PLUS_2; k++) s->word_buff[k] = c->word_buff[k];
    s->frame_lock = c->frame_lock; s->frame_lock_pend = c->frame_lock_pend;
    s->bit_number = c->bit_number; s->subframe = c->subframe;
    s->freq_lock = c->freq_lock; s->freq_lock_ticks = c->freq_lock_ticks;
    const Phase_lock_loop& p = c->aPLL;
    const float pv[17] = {p.PLLBW, p.FLLBW, p.a3, p.b3, p.w0p, p.w0p2, p.w0p3, p.a2, p.w0f,
                          p.w0f2, p.gain, p.w, p.x, p.z, p.pll_lock, 0.0f, p.t};
    memcpy(s->pll, pv, sizeof pv);
    const Delay_lock_loop& d = c->aDLL;
    const float dv[7] = {d.DLLBW, d.x, d.z, d.a, d.w0, d.w02, d.t};
    memcpy(s->dll, dv, sizeof dv);
  }
};

extern "C" {

int ref_chan_state_size(void) { return (int)sizeof(RefChanState); }

void* ref_chan_new(int chan)
{
  static bool piped = false;
  if (!piped) {   // the ephemeris pipe (main/init.cpp:352), read end non-blocking
    if (pipe((int*)CHN_2_EPH_P) == 0) {
      fcntl(CHN_2_EPH_P[READ], F_SETFL, O_NONBLOCK);
      fcntl(CHN_2_EPH_P[WRITE], F_SETPIPE_SZ, 1 << 20);
    }
    piped = true;
  }
  return new Channel(chan);
}

void ref_chan_free(void* c) { delete (Channel*)c; }

void ref_chan_start(void* c, int sv, int doppler, int corr_len)
{
  Acq_Command_S r;
  memset(&r, 0, sizeof r);
  r.sv = sv;
  r.doppler = doppler;
  ((Channel*)c)->Start(sv, r, corr_len);
}

// one Channel::Accum; corr = I[3], Q[3] (E, P, L); fb = NCO_Command_S
void ref_chan_accum(void* c, const int32* corr, NCO_Command_S* fb)
{
  Correlation_S k;
  for (int j = 0; j < 3; j++) { k.I[j] = corr[j]; k.Q[j] = corr[3 + j]; }
  ((Channel*)c)->Accum(&k, fb);
}

void ref_chan_state(void* c, void* out) { Telemetry::get((Channel*)c, (RefChanState*)out); }

// subframes written by ProcessDataBit since the last call; returns the count
int ref_chan_read_subframes(Channel_2_Ephemeris_S* out, int max)
{
  int n = 0;
  while (n < max && read(CHN_2_EPH_P[READ], &out[n], sizeof(Channel_2_Ephemeris_S)) ==
                        (ssize_t)sizeof(Channel_2_Ephemeris_S))
    n++;
  return n;
}

int ref_chan_parity(uint32 word)
{
  Channel* c = new Channel(99);
  const bool ok = c->ParityCheck(word);
  delete c;
  return ok;
}

}  // extern "C"
