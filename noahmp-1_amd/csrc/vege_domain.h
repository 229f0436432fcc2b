// The input domain of the canopy Newton loop's short divisions (sflx_kernel.hip
// vege_flux, DivFast32 in sflx_math.h), and below it the stomata bisection's.
//
// Every division of the loop (vege_flux with its sfcdif1 and ragrb,
// func.f90:2744-2877, :3353-3508, :3260-3350) is exact in the short sequence
// when its operands stay inside DivFast32's exact region.  tools/div_proof.py
// derives, site by site, bounds on both operands and the quotient from the
// limits below, by interval arithmetic in the loop's own order, and checks
// them against that region; DESIGN.md "Division in the canopy loop" records
// the table.  The loop-invariant limits are checked once per column at loop
// entry, the canopy temperature and the ground resistance at every iteration,
// the stomatal resistances after the first; a lane outside any of them repeats
// the loop from its start with IEEE division, so its results are the
// reference's bits either way.  tools/div_proof.py reads this file: it is the
// one copy of the numbers.
#pragma once

// air, ground and canopy temperatures (K); TV at the start of every iteration
#ifndef NMP_DOM_T_LO
#define NMP_DOM_T_LO 150.0
#endif
#ifndef NMP_DOM_T_HI
#define NMP_DOM_T_HI 500.0
#endif
// surface pressure (Pa), vapour pressure of the air (Pa), air density (kg m-3);
// the specific humidity QAIR is checked to lie in [0, 1]
#ifndef NMP_DOM_P_LO
#define NMP_DOM_P_LO 3.0e4
#endif
#ifndef NMP_DOM_P_HI
#define NMP_DOM_P_HI 1.5e5
#endif
#ifndef NMP_DOM_EAIR_HI
#define NMP_DOM_EAIR_HI 1.5e4
#endif
#ifndef NMP_DOM_RHO_LO
#define NMP_DOM_RHO_LO 0.2
#endif
#ifndef NMP_DOM_RHO_HI
#define NMP_DOM_RHO_HI 4.0
#endif
// wind speed UR (m s-1; >= 1 by the reference's own MAX)
#ifndef NMP_DOM_UR_HI
#define NMP_DOM_UR_HI 100.0
#endif
// sfcdif1's log factors log((ZLVL-ZPD)/Z0M) and log((2+Z0H)/Z0H)
#ifndef NMP_DOM_TMPC_LO
#define NMP_DOM_TMPC_LO 0.05
#endif
#ifndef NMP_DOM_TMPC_HI
#define NMP_DOM_TMPC_HI 30.0
#endif
// ZLVL - ZPD (m), canopy height HCAN (m), roughness lengths Z0M, Z0MG (m);
// also ZPD = 0 or in [Z0_LO, HCAN], Z0MG <= HCAN and Z0M + ZPD <= 2 HCAN
#ifndef NMP_DOM_DZ_LO
#define NMP_DOM_DZ_LO 1.0e-2
#endif
#ifndef NMP_DOM_DZ_HI
#define NMP_DOM_DZ_HI 1.0e4
#endif
#ifndef NMP_DOM_HCAN_LO
#define NMP_DOM_HCAN_LO 0.5
#endif
#ifndef NMP_DOM_HCAN_HI
#define NMP_DOM_HCAN_HI 100.0
#endif
#ifndef NMP_DOM_Z0_LO
#define NMP_DOM_Z0_LO 1.0e-5
#endif
#ifndef NMP_DOM_Z0_HI
#define NMP_DOM_Z0_HI 10.0
#endif
// CWP * VAIE * HCAN (ragrb's CWPC = SQRT(CWP*VAI*HCAN*FHG), :3343)
#ifndef NMP_DOM_CWPH_LO
#define NMP_DOM_CWPH_LO 1.0e-3
#endif
#ifndef NMP_DOM_CWPH_HI
#define NMP_DOM_CWPH_HI 50.0
#endif
// canopy area indices (VAIE >= this; LAISUNE / LAISHAE 0 or >= this), wet
// fraction FWET (0 or >= this), vegetated fraction FVEG (>= this)
#ifndef NMP_DOM_VAI_LO
#define NMP_DOM_VAI_LO 1.0e-2
#endif
#ifndef NMP_DOM_LAI_LO
#define NMP_DOM_LAI_LO 1.0e-4
#endif
#ifndef NMP_DOM_FWET_LO
#define NMP_DOM_FWET_LO 1.0e-12
#endif
#ifndef NMP_DOM_FVEG_LO
#define NMP_DOM_FVEG_LO 1.0e-4
#endif
// SQRT(DLEAF/UC) (ragrb :3349), soil surface resistance RSURF (s m-1)
#ifndef NMP_DOM_SDL_LO
#define NMP_DOM_SDL_LO 1.0e-3
#endif
#ifndef NMP_DOM_SDL_HI
#define NMP_DOM_SDL_HI 10.0
#endif
#ifndef NMP_DOM_RSURF_HI
#define NMP_DOM_RSURF_HI 1.0e7
#endif
// stomatal resistances RSSUN, RSSHA (s m-1), after the first iteration
#ifndef NMP_DOM_RS_HI
#define NMP_DOM_RS_HI 1.0e16
#endif
// ground aerodynamic resistance RAHG (s m-1), every iteration
#ifndef NMP_DOM_RAHG_LO
#define NMP_DOM_RAHG_LO 1.0e-3
#endif
#ifndef NMP_DOM_RAHG_HI
#define NMP_DOM_RAHG_HI 1.0e10
#endif
// The per-iteration windows on TV (canopy loop, iterations >= 2) and TGB
// (bare loop) are the temperature limits above.  They have their own names
// only so that a probe build can narrow them alone (-DNMP_DOM_TV_HI=...,
// tests/probe_midloop.py): lanes then leave the domain part way through a
// loop, after it has changed TV/TAH/EAH/QSFC, which exercises the IEEE
// re-run's restore path.  (Not numeric: tools/div_proof.py skips them.)
#ifndef NMP_DOM_TV_HI
#define NMP_DOM_TV_HI NMP_DOM_T_HI
#endif
#ifndef NMP_DOM_TGB_HI
#define NMP_DOM_TGB_HI NMP_DOM_T_HI
#endif
// The numerators of CTR, TR and DTV = B/A (canopy loop) and DTG = B/A (bare
// loop) are products and sums of several possibly small terms that no static
// bound keeps away from the subnormals; with NMP_VD_CHECKED they are checked
// per lane every iteration instead: 0, or 2^NUM_LO_EXP <= |x| <= 2^NUM_HI_EXP
// (a lane outside re-runs its loop with IEEE division).  The ground emissivity
// EMG lies in [0, 1] and the bare loop's CGH = 2*DF/DZ of the top layer in
// [0, CGH_HI], both checked once per column: they bound the denominators A.
#ifndef NMP_DOM_NUM_LO_EXP
#define NMP_DOM_NUM_LO_EXP -96
#endif
#ifndef NMP_DOM_NUM_HI_EXP
#define NMP_DOM_NUM_HI_EXP 64
#endif
#ifndef NMP_DOM_CGH_HI
#define NMP_DOM_CGH_HI 1.0e6
#endif

// ---- the stomata bisection (stomata, func.f90:3739-3887; sflx_kernel.hip
// stomata_solve), run in the canopy loop's first iteration.  Its six divisions
// per bisection step use DivFast32 when, besides the canopy loop's domain
// above, the column's inputs lie in the limits below (checked once, before the
// two calls; a lane outside them runs the bisection with IEEE division) and
// its vegetation type's parameters lie in the box below (checked on the host,
// VegRec::stomata_fast).  tools/div_proof.py proves the sites per 1 K band of
// the canopy temperature.
// absorbed PAR per leaf area, PARSUN / PARSHA (W m-2): <= 0 (no bisection) or in
#ifndef NMP_DOM_APAR_LO
#define NMP_DOM_APAR_LO 1.0e-6
#endif
#ifndef NMP_DOM_APAR_HI
#define NMP_DOM_APAR_HI 1.0e4
#endif
// canopy-air vapour pressure EAH (Pa) at the first iteration: 0 or in
#ifndef NMP_DOM_EAH_LO
#define NMP_DOM_EAH_LO 1.0e-2
#endif
#ifndef NMP_DOM_EAH_HI
#define NMP_DOM_EAH_HI 1.5e4
#endif
// CO2 and O2 partial pressures (Pa)
#ifndef NMP_DOM_CO2_LO
#define NMP_DOM_CO2_LO 1.0
#endif
#ifndef NMP_DOM_CO2_HI
#define NMP_DOM_CO2_HI 1.0e3
#endif
#ifndef NMP_DOM_O2_LO
#define NMP_DOM_O2_LO 1.0e3
#endif
#ifndef NMP_DOM_O2_HI
#define NMP_DOM_O2_HI 1.0e5
#endif
// foliage nitrogen factor FNF = MIN(FOLN / MAX(MPE, FOLNMX), 1): 0 or >= this
#ifndef NMP_DOM_FNF_LO
#define NMP_DOM_FNF_LO 1.0e-3
#endif
// canopy temperature TV at the first iteration (K): <= this (VCMX's
// high-temperature factor 1 + EXP(...) reaches 2e3 at 340 K, 1e14 at 500 K)
#ifndef NMP_DOM_STOMATA_TV_HI
#define NMP_DOM_STOMATA_TV_HI 340.0
#endif
// vegetation-type parameters (VEGPARM.TBL; every shipped table lies inside)
#ifndef NMP_DOM_KC25_LO
#define NMP_DOM_KC25_LO 20.0
#endif
#ifndef NMP_DOM_KC25_HI
#define NMP_DOM_KC25_HI 40.0
#endif
#ifndef NMP_DOM_AKC_LO
#define NMP_DOM_AKC_LO 2.0
#endif
#ifndef NMP_DOM_AKC_HI
#define NMP_DOM_AKC_HI 2.2
#endif
#ifndef NMP_DOM_KO25_LO
#define NMP_DOM_KO25_LO 2.0e4
#endif
#ifndef NMP_DOM_KO25_HI
#define NMP_DOM_KO25_HI 4.0e4
#endif
#ifndef NMP_DOM_AKO_LO
#define NMP_DOM_AKO_LO 1.1
#endif
#ifndef NMP_DOM_AKO_HI
#define NMP_DOM_AKO_HI 1.3
#endif
#ifndef NMP_DOM_AVCMX_LO
#define NMP_DOM_AVCMX_LO 2.3
#endif
#ifndef NMP_DOM_AVCMX_HI
#define NMP_DOM_AVCMX_HI 2.5
#endif
#ifndef NMP_DOM_VCMX25_LO
#define NMP_DOM_VCMX25_LO 1.0
#endif
#ifndef NMP_DOM_VCMX25_HI
#define NMP_DOM_VCMX25_HI 200.0
#endif
#ifndef NMP_DOM_QE25_LO
#define NMP_DOM_QE25_LO 1.0e-3
#endif
#ifndef NMP_DOM_QE25_HI
#define NMP_DOM_QE25_HI 0.2
#endif
#ifndef NMP_DOM_MP_LO
#define NMP_DOM_MP_LO 1.0
#endif
#ifndef NMP_DOM_MP_HI
#define NMP_DOM_MP_HI 20.0
#endif
#ifndef NMP_DOM_BP_LO
#define NMP_DOM_BP_LO 100.0
#endif
#ifndef NMP_DOM_BP_HI
#define NMP_DOM_BP_HI 1.0e16
#endif
// TMIN (K) of a type with VCMX25 > 0: PSN > 0 needs IGS = 1, i.e. TV > TMIN
#ifndef NMP_DOM_TMIN_LO
#define NMP_DOM_TMIN_LO 250.0
#endif
#ifndef NMP_DOM_TMIN_HI
#define NMP_DOM_TMIN_HI 300.0
#endif
