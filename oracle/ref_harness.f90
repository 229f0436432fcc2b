! ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
!
! Batch harness around the reference Fortran `noahmp_sflx`
! (/root/reference/core/module_noahmp_func.f90:66-476).  The reference has no
! caller (its engine slot core/module_noahmp_engine.f90:5-10 is empty), so this
! file plays the role of the offline driver: it owns the per-column state in
! flat arrays, calls `noahmp_sflx` once per column per step, and provides the
! two host externals the reference expects (`wrf_message`, `wrf_error_fatal`,
! called at core/module_noahmp_func.f90:377,708-720,1291,2728-2737,3414,4590).
! Instead of aborting, the externals record a per-column status bitmask (the
! same bits the engine reports, include/noahmp_engine.h NMP_ST_*), and the
! reference simply continues, exactly as it does after the call returns.
!
! Flat layouts (row = one column, C row-major == Fortran (nfield, ncol)):
!   st(56,n)  prognostic fp state, order of NMP_STATE_* in include/noahmp_engine.h
!   isnow(n)  ISNOW
!   sf(6,n)   static fp   (LAT, ZLVL, SHDFAC, SHDMAX, TBOT, FOLN)
!   si(6,n)   static int  (vegtyp, soiltyp, slopetyp, soilcolor, IST, ICE)
!   fc(12,n)  forcing     (SFCTMP SFCPRS PSFC UU VV Q2 SOLDN LWDN PRCP COSZ CO2AIR O2AIR)
!   dg(58,n)  diagnostics, order of NMP_DIAG_* (noahmp_sflx dummy order :82-91)
!   status(n) bitmask
! FICEOLD is derived from the state at step start, as an offline driver does.
module ref_status
  use iso_c_binding
  implicit none
  integer(c_int32_t) :: cur_status = 0
  integer(c_int32_t), parameter :: ST_ERRSW = 1, ST_ERRENG = 2, ST_FIRE = 4, &
       & ST_HCAN = 8, ST_ZLVL = 16, ST_FLERCH = 32, ST_OPTVEG = 64, ST_STOP = 128
  integer :: last_msg_kind = 0
end module ref_status

subroutine wrf_message(msg)
  use ref_status
  implicit none
  character(len=*), intent(in) :: msg
  if (index(msg, 'Flerchinger') > 0) cur_status = ior(cur_status, ST_FLERCH)
  if (index(msg, 'ERRSW') > 0) last_msg_kind = 1
  if (index(msg, 'ERRENG') > 0) last_msg_kind = 2
  if (index(msg, 'HCAN') > 0) last_msg_kind = 3
end subroutine wrf_message

subroutine wrf_error_fatal(msg)
  use ref_status
  implicit none
  character(len=*), intent(in) :: msg
  if (index(msg, 'Stop in Noah-MP') > 0) then
     cur_status = ior(cur_status, ST_ERRSW)
  else if (index(msg, 'energy budget') > 0) then
     cur_status = ior(cur_status, ST_ERRENG)
  else if (index(msg, 'VEGEFLUX') > 0) then
     cur_status = ior(cur_status, ST_HCAN)
  else if (index(msg, 'opt_veg') > 0) then
     cur_status = ior(cur_status, ST_OPTVEG)
  else
     ! 'STOP in Noah-MP' is shared by the FIRE<=0 (:1291) and ZLVL<=ZPD (:3414) checks
     cur_status = ior(cur_status, ST_STOP)
  end if
end subroutine wrf_error_fatal

module ref_harness
  use iso_c_binding
  use noahmp_global
  use noahmp_func, only: noahmp_sflx, frh2o, calhum
  use ref_status
  implicit none
  integer, parameter :: NST = 56, NSF = 6, NSI = 6, NFC = 12, NDG = 58
  real, allocatable :: fice_in(:, :)  ! caller FICEOLD (ref_set_ficeold), else derived
contains

  subroutine ref_set_options(opts) bind(C, name='ref_set_options')
    integer(c_int32_t), intent(in) :: opts(12)
    call noahmp_set_options(opts(1), opts(2), opts(3), opts(4), opts(5), opts(6), &
         & opts(7), opts(8), opts(9), opts(10), opts(11), opts(12))
  end subroutine ref_set_options

  ! Reads the three tables from the current working directory, exactly like
  ! the reference readers do (core/module_noahmp_utils.f90:61).
  subroutine ref_read_tables(soil_tag, slen, veg_tag, vlen) bind(C, name='ref_read_tables')
    use noahmp_gen_param, only: noahmp_gen_param_readptable
    use noahmp_soil_param, only: noahmp_soil_param_readptable
    use noahmp_veg_param, only: noahmp_veg_param_readptable
    integer(c_int32_t), value :: slen, vlen
    character(kind=c_char), intent(in) :: soil_tag(slen), veg_tag(vlen)
    character(len=64) :: st, vt
    integer :: i
    st = ' '
    vt = ' '
    do i = 1, slen
       st(i:i) = soil_tag(i)
    end do
    do i = 1, vlen
       vt(i:i) = veg_tag(i)
    end do
    call noahmp_gen_param_readptable()
    call noahmp_soil_param_readptable(trim(st))
    call noahmp_veg_param_readptable(trim(vt))
  end subroutine ref_read_tables

  ! Dump every table value the physics reads, for pinning the engine's own
  ! TBL parser.  Layout documented in tests/golden/make_golden.py (PARAM_DUMP).
  subroutine ref_dump_params(buf, nbuf, ibuf, nibuf) bind(C, name='ref_dump_params')
    use noahmp_gen_param
    use noahmp_soil_param
    use noahmp_veg_param
    integer(c_int32_t), value :: nbuf, nibuf
    real(c_float), intent(out) :: buf(nbuf)
    integer(c_int32_t), intent(out) :: ibuf(nibuf)
    integer :: k
    k = 0
    call put(LK_SLOPE, MSLOPETYP)
    call put1(KK_CSOIL); call put1(KK_ZBOT); call put1(KK_CZIL); call put1(KK_DKREF)
    call put1(KK_KDTREF); call put1(KK_FRZK); call put1(KK_TIMEAN); call put1(KK_FSATMAX)
    call put1(KK_MLTFCT); call put1(KK_Z0SNO); call put1(KK_SSI); call put1(KK_SWEMAX)
    call put(KK_ALBICE, 2); call put(KK_ALBLAKE, 2); call put(KK_OMEGAS, 2)
    call put1(KK_BETADS); call put1(KK_BETAIS); call put1(KK_EMSSOIL); call put1(KK_EMSLAKE)
    call put(LK_BEXP, MSLTYP); call put(LK_SMCMAX, MSLTYP); call put(LK_SMCREF, MSLTYP)
    call put(LK_SMCWLT, MSLTYP); call put(LK_PSISAT, MSLTYP); call put(LK_DKSAT, MSLTYP)
    call put(LK_DWSAT, MSLTYP); call put(LK_QUARTZ, MSLTYP); call put(LK_KDT, MSLTYP)
    call put(LK_FRZX, MSLTYP)
    call put(reshape(LK_ALBSAT, [2*MSLCOL]), 2*MSLCOL)
    call put(reshape(LK_ALBDRY, [2*MSLCOL]), 2*MSLCOL)
    call put(LK_XL, MLUTYP)
    call put(reshape(LK_RHOL, [2*MLUTYP]), 2*MLUTYP)
    call put(reshape(LK_RHOS, [2*MLUTYP]), 2*MLUTYP)
    call put(reshape(LK_TAUL, [2*MLUTYP]), 2*MLUTYP)
    call put(reshape(LK_TAUS, [2*MLUTYP]), 2*MLUTYP)
    call put(LK_CANWMXP, MLUTYP); call put(LK_DLEAF, MLUTYP); call put(LK_Z0MVT, MLUTYP)
    call put(LK_HVT, MLUTYP); call put(LK_HVB, MLUTYP); call put(LK_DEN, MLUTYP)
    call put(LK_RCROWN, MLUTYP); call put(LK_CWPVT, MLUTYP)
    call put(reshape(LK_SAI12M, [12*MLUTYP]), 12*MLUTYP)
    call put(reshape(LK_LAI12M, [12*MLUTYP]), 12*MLUTYP)
    call put(LK_SLA, MLUTYP); call put(LK_DILEFC, MLUTYP); call put(LK_DILEFW, MLUTYP)
    call put(LK_FRAGR, MLUTYP); call put(LK_LTOVRC, MLUTYP); call put(LK_WRRAT, MLUTYP)
    call put(LK_WDPOOL, MLUTYP); call put(LK_TDLEF, MLUTYP)
    call put(LK_RGL, MLUTYP); call put(LK_HS, MLUTYP); call put(LK_RSMAX, MLUTYP)
    call put(LK_RSMIN, MLUTYP); call put(LK_TOPT, MLUTYP)
    call put(LK_KC25, MLUTYP); call put(LK_AKC, MLUTYP); call put(LK_KO25, MLUTYP)
    call put(LK_AKO, MLUTYP); call put(LK_VCMX25, MLUTYP); call put(LK_AVCMX, MLUTYP)
    call put(LK_BP, MLUTYP); call put(LK_MP, MLUTYP); call put(LK_QE25, MLUTYP)
    call put(LK_AQE, MLUTYP); call put(LK_FOLNMX, MLUTYP); call put(LK_TMIN, MLUTYP)
    call put(LK_RMF25, MLUTYP); call put(LK_RMS25, MLUTYP); call put(LK_RMR25, MLUTYP)
    call put(LK_ARM, MLUTYP); call put(LK_MRP, MLUTYP)
    call put(LK_SLAREA, MLUTYP)
    call put(reshape(LK_EPS, [5*MLUTYP]), 5*MLUTYP)
    ibuf(1) = nslptyp; ibuf(2) = nsltyp; ibuf(3) = nsoilcol; ibuf(4) = nlutyp
    ibuf(5) = ISURBAN; ibuf(6) = ISWATER; ibuf(7) = ISBARREN; ibuf(8) = ISICE; ibuf(9) = ISEGBLF
    ibuf(10:9+MLUTYP) = LK_NROOT(1:MLUTYP)
    ibuf(10+MLUTYP:9+2*MLUTYP) = LK_C3C4(1:MLUTYP)
    ibuf(10+2*MLUTYP) = k
  contains
    subroutine put(a, m)
      integer, intent(in) :: m
      real(c_float), intent(in) :: a(m)
      if (k + m <= nbuf) buf(k+1:k+m) = a(1:m)
      k = k + m
    end subroutine put
    subroutine put1(x)
      real(c_float), intent(in) :: x
      if (k + 1 <= nbuf) buf(k+1) = x
      k = k + 1
    end subroutine put1
  end subroutine ref_dump_params

  ! One noahmp_sflx time step for every column.
  subroutine ref_sflx_batch(n, dt, yearlen, julian, zsoil, st, isnow, sf, si, fc, dg, status) &
       & bind(C, name='ref_sflx_batch')
    integer(c_int32_t), value :: n, yearlen
    real(c_float), value :: dt, julian
    real(c_float), intent(in) :: zsoil(4)
    real(c_float), intent(inout) :: st(NST, n)
    integer(c_int32_t), intent(inout) :: isnow(n)
    real(c_float), intent(in) :: sf(NSF, n)
    integer(c_int32_t), intent(in) :: si(NSI, n)
    real(c_float), intent(in) :: fc(NFC, n)
    real(c_float), intent(out) :: dg(NDG, n)
    integer(c_int32_t), intent(out) :: status(n)
    integer :: c
    do c = 1, n
       call one_column(c, dt, yearlen, julian, zsoil, st(:, c), isnow(c), sf(:, c), si(:, c), &
            & fc(:, c), dg(:, c), status(c))
    end do
  end subroutine ref_sflx_batch

  ! nsteps steps over a forcing cycle fc(:, :, period) with the records kept in
  ! the harness layout between steps (the CPU baseline's timed loop: no
  ! per-step host transposes).  julian advances by dt/86400 per step.
  subroutine ref_sflx_run(n, nsteps, dt, yearlen, julian0, zsoil, st, isnow, sf, si, fc, period, &
       & dg, status) bind(C, name='ref_sflx_run')
    integer(c_int32_t), value :: n, nsteps, yearlen, period
    real(c_float), value :: dt, julian0
    real(c_float), intent(in) :: zsoil(4)
    real(c_float), intent(inout) :: st(NST, n)
    integer(c_int32_t), intent(inout) :: isnow(n)
    real(c_float), intent(in) :: sf(NSF, n)
    integer(c_int32_t), intent(in) :: si(NSI, n)
    real(c_float), intent(in) :: fc(NFC, n, period)
    real(c_float), intent(out) :: dg(NDG, n)
    integer(c_int32_t), intent(out) :: status(n)
    integer :: s
    do s = 0, nsteps - 1
       call ref_sflx_batch(n, dt, yearlen, julian0 + real(s) * dt / 86400.0, zsoil, st, isnow, &
            & sf, si, fc(:, :, mod(s, period) + 1), dg, status)
    end do
  end subroutine ref_sflx_run

  ! Caller-provided FICEOLD (noahmp_sflx's intent(in) argument, func.f90:129):
  ! ref_set_ficeold(f, n) makes the next batches pass f(:, c) for column c
  ! instead of the step-start ice fraction; ref_set_ficeold(NULL, 0) resets.
  subroutine ref_set_ficeold(f, n) bind(C, name='ref_set_ficeold')
    type(c_ptr), value :: f
    integer(c_int32_t), value :: n
    real(c_float), pointer :: fp(:, :)
    if (allocated(fice_in)) deallocate(fice_in)
    if (n > 0 .and. c_associated(f)) then
       call c_f_pointer(f, fp, [3, n])
       allocate(fice_in(3, n))
       fice_in = fp
    end if
  end subroutine ref_set_ficeold

  ! The reference's one public physics routine besides noahmp_sflx, frh2o
  ! (func.f90:4494-4598), called directly: per-routine golden values.
  subroutine ref_frh2o(n, sltyp, tk, smc, sh2o, out, stat) bind(C, name='ref_frh2o')
    integer(c_int32_t), value :: n
    integer(c_int32_t), intent(in) :: sltyp(n)
    real(c_float), intent(in) :: tk(n), smc(n), sh2o(n)
    real(c_float), intent(out) :: out(n)
    integer(c_int32_t), intent(out) :: stat(n)
    integer :: i
    real :: free
    do i = 1, n
       cur_status = 0
       call frh2o(sltyp(i), free, tk(i), smc(i), sh2o(i))
       out(i) = free
       stat(i) = cur_status
    end do
  end subroutine ref_frh2o

  ! calhum (func.f90:3958-3984): a module procedure of noahmp_func, public by
  ! default (the module's private list does not name it), called directly.
  subroutine ref_calhum(n, sfctmp, sfcprs, q2sat, dqsdt2) bind(C, name='ref_calhum')
    integer(c_int32_t), value :: n
    real(c_float), intent(in) :: sfctmp(n), sfcprs(n)
    real(c_float), intent(out) :: q2sat(n), dqsdt2(n)
    integer :: i
    do i = 1, n
       call calhum(sfctmp(i), sfcprs(i), q2sat(i), dqsdt2(i))
    end do
  end subroutine ref_calhum

  subroutine one_column(c, dt, yearlen, julian, zsoil_in, s, isn, sf, si, fc, d, stat)
    integer, intent(in) :: c, yearlen
    real, intent(in) :: dt, julian
    real, intent(in) :: zsoil_in(4)
    real, intent(inout) :: s(NST)
    integer, intent(inout) :: isn
    real, intent(in) :: sf(NSF), fc(NFC)
    integer, intent(in) :: si(NSI)
    real, intent(out) :: d(NDG)
    integer(c_int32_t), intent(out) :: stat
    real :: zsoil(4), ficeold(-2:0)
    real :: stc(-2:4), zsnso(-2:4), snice(-2:0), snliq(-2:0), sh2o(4), smc(4)
    real :: lat, zlvl, shdfac, shdmax, tbot, foln
    real :: sfctmp, sfcprs, psfc, uu, vv, q2, soldn, lwdn, prcp, cosz, co2air, o2air
    real :: tv, tg, tah, eah, fwet, canliq, canice, qsfc, snowh, sneqv, sneqvo, albold, tauss
    real :: qsnow, zwt, wa, wt, wslake, lai, sai, lfmass, rtmass, stmass, wood, stblcp, fastcp
    real :: cm, ch
    real :: dx, dz8w, qc, pblh
    integer :: iz
    real :: o(NDG)

    zsoil = zsoil_in
    stc = s(1:7); zsnso = s(8:14); snice = s(15:17); snliq = s(18:20)
    sh2o = s(21:24); smc = s(25:28)
    tv = s(29); tg = s(30); tah = s(31); eah = s(32); fwet = s(33); canliq = s(34)
    canice = s(35); qsfc = s(36); snowh = s(37); sneqv = s(38); sneqvo = s(39)
    albold = s(40); tauss = s(41); qsnow = s(42); zwt = s(43); wa = s(44); wt = s(45)
    wslake = s(46); lai = s(47); sai = s(48); lfmass = s(49); rtmass = s(50)
    stmass = s(51); wood = s(52); stblcp = s(53); fastcp = s(54); cm = s(55); ch = s(56)
    lat = sf(1); zlvl = sf(2); shdfac = sf(3); shdmax = sf(4); tbot = sf(5); foln = sf(6)
    sfctmp = fc(1); sfcprs = fc(2); psfc = fc(3); uu = fc(4); vv = fc(5); q2 = fc(6)
    soldn = fc(7); lwdn = fc(8); prcp = fc(9); cosz = fc(10); co2air = fc(11); o2air = fc(12)
    dx = 1000.0; dz8w = 20.0; qc = 0.0; pblh = 1000.0

    ficeold = 0.0
    do iz = isn + 1, 0
       ficeold(iz) = snice(iz) / (snice(iz) + snliq(iz))
    end do
    if (allocated(fice_in)) ficeold = fice_in(:, c)

    cur_status = 0
    o = 0.0
    call noahmp_sflx(c, 1, lat, yearlen, julian, cosz, &
         & dt, dx, dz8w, 4, zsoil, 3, &
         & shdfac, shdmax, si(3), si(2), si(1), si(6), si(5), &
         & si(4), &
         & 0, &
         & sfctmp, sfcprs, psfc, uu, vv, q2, &
         & qc, soldn, lwdn, prcp, tbot, co2air, &
         & o2air, foln, ficeold, pblh, zlvl, &
         & albold, sneqvo, &
         & stc, sh2o, smc, tah, eah, fwet, &
         & canliq, canice, tv, tg, qsfc, qsnow, &
         & isn, zsnso, snowh, sneqv, snice, snliq, &
         & zwt, wa, wt, wslake, lfmass, rtmass, &
         & stmass, wood, stblcp, fastcp, lai, sai, &
         & cm, ch, tauss, &
         & o(1), o(2), o(3), o(4), o(5), o(6), &
         & o(7), o(8), o(9), o(10), o(11), o(12), &
         & o(13), o(14), o(15), o(16), o(17), o(18), &
         & o(19), o(20), o(21), o(22), o(23), o(24), &
         & o(25), o(26), o(27), o(28), o(29), o(30), &
         & o(31), o(32), o(33), o(34), o(35), o(36), &
         & o(37), o(38), o(39), o(40), o(41), &
         & o(42), o(43), o(44), o(45), o(46), o(47), &
         & o(48), o(49), o(50), o(51), o(52), o(53), &
         & o(54), o(55), o(56), o(57), o(58))
    d = o
    stat = cur_status

    s(1:7) = stc; s(8:14) = zsnso; s(15:17) = snice; s(18:20) = snliq
    s(21:24) = sh2o; s(25:28) = smc
    s(29) = tv; s(30) = tg; s(31) = tah; s(32) = eah; s(33) = fwet; s(34) = canliq
    s(35) = canice; s(36) = qsfc; s(37) = snowh; s(38) = sneqv; s(39) = sneqvo
    s(40) = albold; s(41) = tauss; s(42) = qsnow; s(43) = zwt; s(44) = wa; s(45) = wt
    s(46) = wslake; s(47) = lai; s(48) = sai; s(49) = lfmass; s(50) = rtmass
    s(51) = stmass; s(52) = wood; s(53) = stblcp; s(54) = fastcp; s(55) = cm; s(56) = ch
  end subroutine one_column
end module ref_harness
