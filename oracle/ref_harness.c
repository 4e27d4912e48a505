/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Host-side glue that lets the UNMODIFIED reference OSGPS correlator
 * (osgnss_next_step/src/correlator/correlator.c + gp2021/gp2021.c +
 *  isr/osgpsisr.c, compiled by oracle/Makefile straight from /root/reference
 *  into oracle/_ref/) be driven from Python (ctypes) to produce golden vectors.
 *
 * The reference keeps its receiver globals in include/globals.h behind
 * `#define MAIN` (osgnss_next_step.c:1-2 of the main program defines them);
 * this file plays the role of that main translation unit so the reference
 * objects link, and adds two tiny accessors.
 */
#define MAIN
#include "globals.h"

/* correlator.h defines these as tentative definitions (needs -fcommon). */
extern int REG_read[256], REG_write[256];

/* osgpsisr.c writes DEBUG_TRACKING vectors to corr_out; point it at /dev/null
 * so the end-to-end receiver harness can run the unmodified ISR. */
void ref_harness_open_debug(void)
{
  if (!corr_out) corr_out = fopen("/dev/null", "w");
}

/* Byte size of the reference's tracking_channel struct (structs.h:86-128), so
 * Python can walk chan[] without restating the layout. */
int ref_harness_sizeof_tracking_channel(void) { return (int)sizeof(tracking_channel); }
