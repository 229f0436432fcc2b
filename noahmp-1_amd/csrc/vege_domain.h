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
#define NMP_DOM_T_LO 150.0
#define NMP_DOM_T_HI 500.0
// surface pressure (Pa), vapour pressure of the air (Pa), air density (kg m-3);
// the specific humidity QAIR is checked to lie in [0, 1]
#define NMP_DOM_P_LO 3.0e4
#define NMP_DOM_P_HI 1.5e5
#define NMP_DOM_EAIR_HI 1.5e4
#define NMP_DOM_RHO_LO 0.2
#define NMP_DOM_RHO_HI 4.0
// wind speed UR (m s-1; >= 1 by the reference's own MAX)
#define NMP_DOM_UR_HI 100.0
// sfcdif1's log factors log((ZLVL-ZPD)/Z0M) and log((2+Z0H)/Z0H)
#define NMP_DOM_TMPC_LO 0.05
#define NMP_DOM_TMPC_HI 30.0
// ZLVL - ZPD (m), canopy height HCAN (m), roughness lengths Z0M, Z0MG (m);
// also ZPD = 0 or in [Z0_LO, HCAN], Z0MG <= HCAN and Z0M + ZPD <= 2 HCAN
#define NMP_DOM_DZ_LO 1.0e-2
#define NMP_DOM_DZ_HI 1.0e4
#define NMP_DOM_HCAN_LO 0.5
#define NMP_DOM_HCAN_HI 100.0
#define NMP_DOM_Z0_LO 1.0e-5
#define NMP_DOM_Z0_HI 10.0
// CWP * VAIE * HCAN (ragrb's CWPC = SQRT(CWP*VAI*HCAN*FHG), :3343)
#define NMP_DOM_CWPH_LO 1.0e-3
#define NMP_DOM_CWPH_HI 50.0
// canopy area indices (VAIE >= this; LAISUNE / LAISHAE 0 or >= this), wet
// fraction FWET (0 or >= this), vegetated fraction FVEG (>= this)
#define NMP_DOM_VAI_LO 1.0e-2
#define NMP_DOM_LAI_LO 1.0e-4
#define NMP_DOM_FWET_LO 1.0e-12
#define NMP_DOM_FVEG_LO 1.0e-4
// SQRT(DLEAF/UC) (ragrb :3349), soil surface resistance RSURF (s m-1)
#define NMP_DOM_SDL_LO 1.0e-3
#define NMP_DOM_SDL_HI 10.0
#define NMP_DOM_RSURF_HI 1.0e7
// stomatal resistances RSSUN, RSSHA (s m-1), after the first iteration
#define NMP_DOM_RS_HI 1.0e16
// ground aerodynamic resistance RAHG (s m-1), every iteration
#define NMP_DOM_RAHG_LO 1.0e-3
#define NMP_DOM_RAHG_HI 1.0e10

// ---- the stomata bisection (stomata, func.f90:3739-3887; sflx_kernel.hip
// stomata_solve), run in the canopy loop's first iteration.  Its six divisions
// per bisection step use DivFast32 when, besides the canopy loop's domain
// above, the column's inputs lie in the limits below (checked once, before the
// two calls; a lane outside them runs the bisection with IEEE division) and
// its vegetation type's parameters lie in the box below (checked on the host,
// VegRec::stomata_fast).  tools/div_proof.py proves the sites per 1 K band of
// the canopy temperature.
// absorbed PAR per leaf area, PARSUN / PARSHA (W m-2): <= 0 (no bisection) or in
#define NMP_DOM_APAR_LO 1.0e-6
#define NMP_DOM_APAR_HI 1.0e4
// canopy-air vapour pressure EAH (Pa) at the first iteration: 0 or in
#define NMP_DOM_EAH_LO 1.0e-2
#define NMP_DOM_EAH_HI 1.5e4
// CO2 and O2 partial pressures (Pa)
#define NMP_DOM_CO2_LO 1.0
#define NMP_DOM_CO2_HI 1.0e3
#define NMP_DOM_O2_LO 1.0e3
#define NMP_DOM_O2_HI 1.0e5
// foliage nitrogen factor FNF = MIN(FOLN / MAX(MPE, FOLNMX), 1): 0 or >= this
#define NMP_DOM_FNF_LO 1.0e-3
// canopy temperature TV at the first iteration (K): <= this (VCMX's
// high-temperature factor 1 + EXP(...) reaches 2e3 at 340 K, 1e14 at 500 K)
#define NMP_DOM_STOMATA_TV_HI 340.0
// vegetation-type parameters (VEGPARM.TBL; every shipped table lies inside)
#define NMP_DOM_KC25_LO 20.0
#define NMP_DOM_KC25_HI 40.0
#define NMP_DOM_AKC_LO 2.0
#define NMP_DOM_AKC_HI 2.2
#define NMP_DOM_KO25_LO 2.0e4
#define NMP_DOM_KO25_HI 4.0e4
#define NMP_DOM_AKO_LO 1.1
#define NMP_DOM_AKO_HI 1.3
#define NMP_DOM_AVCMX_LO 2.3
#define NMP_DOM_AVCMX_HI 2.5
#define NMP_DOM_VCMX25_LO 1.0
#define NMP_DOM_VCMX25_HI 200.0
#define NMP_DOM_QE25_LO 1.0e-3
#define NMP_DOM_QE25_HI 0.2
#define NMP_DOM_MP_LO 1.0
#define NMP_DOM_MP_HI 20.0
#define NMP_DOM_BP_LO 100.0
#define NMP_DOM_BP_HI 1.0e16
// TMIN (K) of a type with VCMX25 > 0: PSN > 0 needs IGS = 1, i.e. TV > TMIN
#define NMP_DOM_TMIN_LO 250.0
#define NMP_DOM_TMIN_HI 300.0
