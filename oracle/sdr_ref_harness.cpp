// oracle/sdr_ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// C entry points over the GPS-SDR primitives compiled from the reference's own
// sources with -DNO_SIMD (simd/x86.cpp, objects/fft.cpp, accessories/misc.cpp;
// recipe in oracle/Makefile, output only in oracle/_ref/).  The Acquisition
// class itself does not build here (usrp / libusb headers, i386 asm: SURVEY 8c),
// so ref_sdr_acq_strong composes the same calls in the same order as
// Acquisition::doPrepIF (acquisition.cpp:191-236, 1 ms) and doAcqStrong
// (acquisition.cpp:244-301), with the x86_* (wrapping) primitives standing in
// for the production sse_* ones (equal outside int16 saturation).
#include "includes.h"
#include "fft.h"
#include "prn_codes.h"

extern "C" {

void ref_sdr_sine_gen(CPX* dst, double f, double fs, int n) { sine_gen(dst, f, fs, n); }

void ref_sdr_fft(CPX* x, int n, const int32* scale16, int inverse)
{
  int32 r[MAX_RANKS];
  for (int k = 0; k < MAX_RANKS; k++) r[k] = scale16[k];
  FFT f(n, r);
  if (inverse) f.doiFFT(x, true);
  else f.doFFT(x, true);
}

void ref_sdr_cmulsc(CPX* a, CPX* b, CPX* c, int n, int shift) { x86_cmulsc(a, b, c, n, shift); }

void ref_sdr_cmag_max(CPX* a, int n, int32* index, int32* mag)
{
  x86_cmag(a, n);
  x86_max((int32*)a, index, mag, n);
}

const int16* ref_sdr_prn_codes(void) { return PRN_Codes; }

// downsample (accessories/misc.cpp:174-197) from the reference build; returns
// the kept count the same way the reference loop does
int ref_sdr_downsample(CPX* dest, CPX* source, double fdest, double fsource, int samps)
{
  downsample(dest, source, fdest, fsource, samps);
  uint32 step = (uint32)floor((double)4294967296.0 * fdest / fsource), lphase = 0, phase = 0;
  int k = 0;
  for (int lcv = 0; lcv < samps; lcv++) {
    if (phase <= lphase) k++;
    lphase = phase;
    phase += step;
  }
  return k;
}

// code_gen (accessories/misc.cpp:28-87): out[k] = chip (0/1) of sv
void ref_sdr_code_gen(int sv, int16* out)
{
  CPX tmp[1023];
  code_gen(tmp, sv);
  for (int k = 0; k < 1023; k++) out[k] = tmp[k].i;
}

// Correlator::Accum (correlator.cpp:425-448) over the x86 primitives: wipe-off
// then prn_accum_new.  codes: +-1 per sample for E, P, L; out: E.i E.q P.i P.q L.i L.q
void ref_sdr_accum(CPX* data, CPX* sine, const int8_t* e, const int8_t* p, const int8_t* l,
                   int samps, int32* out)
{
  CPX* scratch = new CPX[samps > 0 ? samps : 1];
  MIX* m[3];
  const int8_t* src[3] = {e, p, l};
  for (int j = 0; j < 3; j++) {
    m[j] = new MIX[samps > 0 ? samps : 1];
    for (int k = 0; k < samps; k++) {
      const short v = src[j][k] > 0 ? 0x0001 : (short)0xffff;   // SamplePRN mapping
      m[j][k].i = m[j][k].ni = v;
      m[j][k].q = m[j][k].nq = 0;
    }
  }
  x86_cmulsc(data, sine, scratch, samps, 14);
  CPX_ACCUM epl[3];
  x86_prn_accum_new(scratch, m[0], m[1], m[2], samps, epl);
  for (int j = 0; j < 3; j++) {
    out[2 * j] = epl[j].i;
    out[2 * j + 1] = epl[j].q;
    delete[] m[j];
  }
  delete[] scratch;
}

// out: sv, code_phase, doppler, magnitude, success, row
void ref_sdr_acq_strong(const CPX* buff, double fif, int sv, int doppmin, int doppmax, int32* out)
{
  const int n = SAMPS_MS;
  int32 R1[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int32 R2[16] = {0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 1};
  FFT fwd(n, R1), inv(n, R2);
  CPX* wipe[4];
  for (int j = 0; j < 4; j++) {
    wipe[j] = new CPX[n];
    sine_gen(wipe[j], -fif - 250.0 * j, SAMPLE_FREQUENCY, n);
  }
  CPX* baseband = new CPX[4 * n];
  memcpy(baseband, buff, n * sizeof(CPX));
  for (int j = 1; j < 4; j++) x86_cmulsc(baseband, wipe[j], &baseband[j * n], n, 14);
  x86_cmuls(baseband, wipe[0], n, 14);
  for (int j = 0; j < 4; j++) fwd.doFFT(&baseband[j * n], true);
  CPX* rows = new CPX[4 * (n + 201)];
  for (int j = 0; j < 4; j++) {
    CPX* p = &rows[j * (n + 201)];
    memcpy(p, &baseband[(j + 1) * n - 100], 100 * sizeof(CPX));
    memcpy(p + 100, &baseband[j * n], n * sizeof(CPX));
    memcpy(p + 100 + n, &baseband[j * n], 100 * sizeof(CPX));
  }
  CPX* code = (CPX*)&PRN_Codes[2 * sv * n];
  CPX* msbuff = new CPX[n];
  int32 mag = 0, magt, indext;
  int32 res[6] = {sv, 0, 0, 0, 0, 0};
  for (int lcv = doppmin / 1000; lcv < doppmax / 1000; lcv++)
    for (int lcv2 = 0; lcv2 < 4; lcv2++) {
      x86_cmulsc(&rows[lcv2 * (n + 201) + 100 + lcv], code, msbuff, n, 10);
      inv.doiFFT(msbuff, true);
      x86_cmag(msbuff, n);
      x86_max((int32*)msbuff, &indext, &magt, n);
      if (magt > mag) {
        mag = magt;
        res[1] = 2048 - indext;
        res[2] = (int32)((lcv * 1000) + (float)lcv2 * 250);
        res[3] = mag;
        res[5] = (lcv - doppmin / 1000) * 4 + lcv2;
      }
    }
  res[4] = (uint32)res[3] > THRESH_STRONG ? 1 : 0;
  memcpy(out, res, sizeof res);
  delete[] msbuff;
  delete[] rows;
  delete[] baseband;
  for (int j = 0; j < 4; j++) delete[] wipe[j];
}

}  // extern "C"
