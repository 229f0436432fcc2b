/*
 * ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
 *
 * Plain-C restatement of the reference noahmp_sflx
 * (/root/reference/core/module_noahmp_func.f90:66-476) used as a CPU checker
 * and CPU baseline.  Compiled twice: ORACLE_REAL=float (bit-level follower of
 * the fp32 reference) and ORACLE_REAL=double.  Table layout and option struct
 * come from the public boundary header include/noahmp_engine.h.
 *
 * Layout is the reference harness's (oracle/ref_harness.f90): row per column,
 * st[n][56], sf[n][6], si[n][6], fc[n][12], dg[n][58].
 */
#ifndef NOAHMP_ORACLE_H
#define NOAHMP_ORACLE_H
#include <stdint.h>
#include "../include/noahmp_engine.h"

#ifndef ORACLE_REAL
#define ORACLE_REAL float
#endif

#ifdef __cplusplus
extern "C" {
#endif

int oracle_real_bytes(void);

/* One step over n columns; returns 0. */
int oracle_sflx_batch(int32_t n, ORACLE_REAL dt, int32_t yearlen, ORACLE_REAL julian,
                      const ORACLE_REAL zsoil[4], ORACLE_REAL* st, int32_t* isnow,
                      const ORACLE_REAL* sf, const int32_t* si, const ORACLE_REAL* fc,
                      ORACLE_REAL* dg, int32_t* status, const nmp_params* P,
                      const nmp_options* O);

/* nsteps steps of the same column set, forcing fc[s][n][12]; diag of the last
 * step; used for the timed CPU baseline (nthreads via OpenMP when built so). */
int oracle_sflx_run(int32_t n, int32_t nsteps, ORACLE_REAL dt, int32_t yearlen,
                    ORACLE_REAL julian0, const ORACLE_REAL zsoil[4], ORACLE_REAL* st,
                    int32_t* isnow, const ORACLE_REAL* sf, const int32_t* si,
                    const ORACLE_REAL* fc, int32_t fc_period, ORACLE_REAL* dg, int32_t* status,
                    const nmp_params* P, const nmp_options* O);

#ifdef __cplusplus
}
#endif
#endif
