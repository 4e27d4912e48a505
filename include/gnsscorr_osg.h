/*
 * gnsscorr_osg.h -- drop-in replacement for the OSGPS software-correlator
 * interface (reference: trunk/GNSS_SOFTWARE_RECEIVERS/POSTPROCESSING_RECEIVERS/
 * osgnss_next_step/src/correlator/correlator.h:1-9).
 *
 * Link the reference host side (gp2021/gp2021.c register accessors,
 * isr/osgpsisr.c DLL/PLL state machine, osgnss_next_step.c main loop) against
 * libgnsscorr.so instead of correlator.c; nothing else changes.  The
 * correlation itself runs on the GPU (HIP, gfx950).
 *
 *  correlator_init   replaces correlator.c:107-132
 *  Sim_GP2021_int    replaces correlator.c:148-316 (synchronous: the IF buffer
 *                    is copied to the device before the call returns and the
 *                    REG_read latches are updated before it returns, so the
 *                    caller may reuse IF exactly as osgnss_next_step.c:115 does)
 *  REG_read/REG_write  the GP2021 register file, same types and map
 *                    (correlator.c:9-20).  The reference defines them in its
 *                    header (tentative definitions, -fcommon); this library
 *                    defines them once and exports them.
 *
 * The reference has no error channel (void returns).  On a device error this
 * shim prints the HIP error and calls abort(); on a PRN > 32 (the reference
 * would index past its 33-row tables) it prints and aborts too.
 * `write_to_file_prn_codes` (declared at correlator.h:7) is not exported: the
 * reference never defines it.
 */
#ifndef GNSSCORR_OSG_H
#define GNSSCORR_OSG_H

#ifdef __cplusplus
extern "C" {
#endif

extern int REG_read[256], REG_write[256];

void correlator_init(double tic_period);
void Sim_GP2021_int(char *IF, long nsamp);

/* Receiver globals that the reference's correlator_init() computes
 * (correlator.c:110-125; declared in include/globals.h:41-49).  Defined by
 * this library; when the host program also defines them (globals.h with
 * MAIN), the host's definitions take precedence and are the ones written. */
extern double Carrier_DCO_Delta, Code_DCO_Delta;
extern long gps_code_ref, gps_carrier_ref, glonass_code_ref, glonass_carrier_ref, d_freq;

/* Optional runtime configuration (the reference hard-codes these as
 * #defines in include/globals.h:7-23).  Call before correlator_init().
 * Defaults: fs 16.0e6, GPS IF 2.42e6, GLONASS IF 0, sys clock mult 5,
 * carrier/code NCO widths 30/29, 12 channels, IQ input, 1000 Hz bin width,
 * device 0.  Environment overrides: GNSSCORR_SAMP_RATE, GNSSCORR_IF,
 * GNSSCORR_DEVICE.  Returns 0 or a negative GNSSCORR_E* code. */
int gnsscorr_osg_configure(double samp_rate, double gps_if, double glonass_if,
                           double sys_clock_mult, int carrier_nco_bits, int code_nco_bits,
                           int n_channels, int use_iq, double freq_bin_width, int device);

/* Snapshot of the n_channels correlator channel states (struct gp2021_channel,
 * correlator.c:36-47, plus ms/bit counters) for checkpoint or inspection. */
int gnsscorr_osg_get_state(void *h_state /* gnsscorr_chan_state[n_channels] */);

#ifdef __cplusplus
}
#endif
#endif
