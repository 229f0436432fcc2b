// The input domain of the canopy Newton loop's short divisions (sflx_kernel.hip
// vege_flux, DivFast32 in sflx_math.h).
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
