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
// ref_sdr_acq_session / _prep / _medium / _weak do the same for doPrepIF at
// 10 and 310 ms, doAcqMedium (acquisition.cpp:309-425) and doAcqWeak
// (acquisition.cpp:433-570), over a session holding the object's members.
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

// ---- medium / weak acquisition over the reference primitives --------------
// A session holds the Acquisition members that persist between requests
// (acquisition.cpp:95-142): the 310-ms baseband, the padded baseband_rows
// store of 1240 rows x (2048 + 201), the 10-ms wipe-offs copied 31 times and
// the 10 x 10 post-correlation DFT rows.  The reference allocates the rows
// with new[] (no value initialisation); calloc stands in for the zero pages
// such a 22 MB allocation gets from a fresh mmap.
struct RefAcqSession {
  CPX *baseband, *shift, *wipe[4], *coherent, *power;
  CPX **rows;
  MIX *dft, *dft_rows[10];
  FFT *fwd, *inv;
  double fif;
};

void* ref_sdr_acq_session(double fif)
{
  const int n = SAMPS_MS;
  int32 R1[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int32 R2[16] = {0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 1};
  RefAcqSession* s = new RefAcqSession;
  s->fif = fif;
  s->baseband = (CPX*)calloc((size_t)4 * 310 * n, sizeof(CPX));
  s->shift = (CPX*)calloc((size_t)4 * 310 * (n + 201), sizeof(CPX));
  s->rows = new CPX*[1240];
  for (int k = 0; k < 1240; k++) s->rows[k] = &s->shift[(size_t)k * (n + 201)];
  s->coherent = new CPX[10 * n];
  s->power = new CPX[10 * n];
  s->dft = new MIX[100];
  for (int k = 0; k < 10; k++) {
    s->dft_rows[k] = &s->dft[k * 10];
    wipeoff_gen(s->dft_rows[k], (float)k * 25.0 - 112.5, 1000.0, 10);
  }
  for (int j = 0; j < 4; j++) {
    s->wipe[j] = new CPX[310 * n];
    sine_gen(s->wipe[j], -fif - 250.0 * j, SAMPLE_FREQUENCY, 10 * n);
    for (int k = 1; k < 31; k++) memcpy(&s->wipe[j][k * 10 * n], s->wipe[j], 10 * n * sizeof(CPX));
  }
  s->fwd = new FFT(n, R1);
  s->inv = new FFT(n, R2);
  return s;
}

void ref_sdr_acq_session_free(void* p)
{
  RefAcqSession* s = (RefAcqSession*)p;
  free(s->baseband);
  free(s->shift);
  delete[] s->rows;
  delete[] s->coherent;
  delete[] s->power;
  delete[] s->dft;
  for (int j = 0; j < 4; j++) delete[] s->wipe[j];
  delete s->fwd;
  delete s->inv;
  delete s;
}

// doPrepIF (acquisition.cpp:191-236), ms = 1, 10 or 310
void ref_sdr_acq_prep(void* p, const CPX* buff, int ms)
{
  RefAcqSession* s = (RefAcqSession*)p;
  const int n = SAMPS_MS;
  memcpy(s->baseband, buff, (size_t)ms * n * sizeof(CPX));
  for (int j = 1; j < 4; j++)
    x86_cmulsc(&s->baseband[0], s->wipe[j], &s->baseband[(size_t)j * ms * n], ms * n, 14);
  x86_cmuls(s->baseband, s->wipe[0], ms * n, 14);
  for (int k = 0; k < 4 * ms; k++) s->fwd->doFFT(&s->baseband[(size_t)k * n], true);
  for (int k = 0; k < 4 * ms; k++) {
    CPX* r = s->rows[k];
    memcpy(r, &s->baseband[(size_t)(k + 1) * n - 100], 100 * sizeof(CPX));
    memcpy(r + 100, &s->baseband[(size_t)k * n], n * sizeof(CPX));
    memcpy(r + 100 + n, &s->baseband[(size_t)k * n], 100 * sizeof(CPX));
  }
}

// the 1-ms-block post-correlation DFT of one delay column (acquisition.cpp:350-373)
static void ref_post_dft(RefAcqSession* s, int col, CPX temp[10])
{
  const int n = SAMPS_MS;
  int32 data[32];
  int32* q = (int32*)&s->coherent[col];
  for (int m = 0; m < 10; m++) { data[m] = *q; q += n; }
  for (int j = 0; j < 10; j++) {
    int32 ia, qa;
    x86_cacc((CPX*)data, s->dft_rows[j], 10, &ia, &qa);
    temp[j].i = ia >> 16;
    temp[j].q = qa >> 16;
  }
}

// out: sv, code_phase, doppler, magnitude, success, row  (acquisition.cpp:309-425)
void ref_sdr_acq_medium(void* p, int sv, int doppmin, int doppmax, int32* out)
{
  RefAcqSession* s = (RefAcqSession*)p;
  const int n = SAMPS_MS;
  CPX* code = (CPX*)&PRN_Codes[2 * sv * n];
  int32 mag = 0, magt, indext, res[6] = {sv, 0, 0, 0, 0, 0};
  for (int lcv = doppmin / 1000; lcv <= doppmax / 1000; lcv++)
    for (int lcv2 = 0; lcv2 < 4; lcv2++) {
      const int k = 0;
      for (int l3 = 0; l3 < 10; l3++) {
        x86_cmulsc(&s->rows[lcv2 * 20 + l3 + k * 10][100 + lcv], code, &s->coherent[l3 * n], n, 10);
        s->inv->doiFFT(&s->coherent[l3 * n], true);
      }
      for (int l3 = 0; l3 < n; l3++) {
        CPX temp[10];
        ref_post_dft(s, l3, temp);
        int32* q = (int32*)&s->power[l3];
        for (int j = 0; j < 10; j++) { *q = *(int32*)&temp[j]; q += n; }
      }
      x86_cmag(&s->power[0], 10 * n);
      x86_max((int32*)s->power, &indext, &magt, 10 * n);
      if (magt > mag) {
        mag = magt;
        res[1] = indext % n;
        res[2] = (lcv * 1000) + (lcv2 * 250) + (indext / n) * 25.0;
        res[3] = mag;
        res[5] = (lcv - doppmin / 1000) * 4 + lcv2;
      }
    }
  res[4] = (uint32)res[3] > THRESH_MEDIUM ? 1 : 0;
  memcpy(out, res, sizeof res);
}

// out: sv, code_phase, doppler, magnitude, success, row  (acquisition.cpp:433-570)
void ref_sdr_acq_weak(void* p, int sv, int doppmin, int doppmax, int32* out)
{
  RefAcqSession* s = (RefAcqSession*)p;
  const int n = SAMPS_MS;
  CPX* code = (CPX*)&PRN_Codes[2 * sv * n];
  int32 mag = 0, magt, indext, res[6] = {sv, 0, 0, 0, 0, 0};
  for (int lcv = doppmin / 1000; lcv < doppmax / 1000; lcv++)
    for (int lcv2 = 0; lcv2 < 4; lcv2++)
      for (int k = 0; k < 2; k++) {
        memset(s->power, 0x0, 10 * n * sizeof(CPX));
        for (int i = 0; i < 15; i++) {
          for (int l3 = 0; l3 < 10; l3++) {
            x86_cmulsc(&s->rows[lcv2 * 310 + l3 + i * 20 + k * 10][100 + lcv], code,
                       &s->coherent[l3 * n], n, 9);
            s->inv->doiFFT(&s->coherent[l3 * n], true);
          }
          double doppler = (double)(lcv * 1000) + (float)(lcv2 * 250);
          double code_doppler = (double)i * .02 * IF_SAMPLE_FREQUENCY * doppler / L1;
          int32 shift = (int32)floor(code_doppler);
          for (int l3 = 0; l3 < n; l3++) {
            CPX temp[10];
            ref_post_dft(s, l3, temp);
            x86_cmag(&temp[0], 10);
            int32* q = (int32*)&s->power[(l3 + shift + SAMPS_MS) % SAMPS_MS];
            for (int j = 0; j < 10; j++) { *q += ((int32*)temp)[j]; q += n; }
          }
        }
        x86_max((int32*)s->power, &indext, &magt, 10 * n);
        if (magt > mag) {
          mag = magt;
          res[1] = indext % n;
          res[2] = (lcv * 1000) + (lcv2 * 250) + (indext / n) * 25.0;
          res[3] = mag;
          res[5] = ((lcv - doppmin / 1000) * 4 + lcv2) * 2 + k;
        }
      }
  res[4] = (uint32)res[3] > THRESH_WEAK ? 1 : 0;
  memcpy(out, res, sizeof res);
}

}  // extern "C"
