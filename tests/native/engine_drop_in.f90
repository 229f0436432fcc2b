! The Fortran engine slot of INTEGRATION.md, exercised at run time.  The module
! `noahmp_engine` (extracted verbatim from INTEGRATION.md by
! __graft_entry__.build()) replaces the reference's empty engine slot
! (core/module_noahmp_engine.f90:5-10).  This program drives it the way a
! Fortran host of the reference would: options through the reference's own
! noahmp_set_options (module noahmp_global, compiled from /root/reference by
! oracle/Makefile), then either
!   mode "run" : noahmp_init once, noahmp_run every step over the module's
!                column arrays (state resident on the device), or
!   mode "runl": as "run", with the step's LDASIN block (nmp_ldasin, taken
!                from the forcing's T2D Q2D U2D V2D PSFC RAINRATE SWDOWN LWDOWN
!                COSZ) and nmp_ldasin_forcing, the forcing formed on the device;
!   mode "runc": as "runl", on forcing whose 8 LDASIN variables hold over
!                groups of 4 steps: steps 2-4 of a group upload only COSZ
!                (nmp_ldasin_cosz_only);
!   mode "sflx": one noahmp_sflx call per column per step with the
!                reference's 131 arguments (FICEOLD from the step-start ice
!                fraction, as the reference harness passes it).
! tests/test_gpu_routines.py compares every step with the reference trajectory.
!
! Mode "time" (profiles/, DESIGN.md "The Fortran slot timed"): the fixture's
! columns replicated to <ncol> columns, <nsteps> timed noahmp_run calls after
! 2 untimed ones, diagnostics (level 1, the 16 output fluxes) copied back on
! every <out_every>-th step and level 0 otherwise, arrays page-locked or not
! (<pinned> 1|0).  Writes one line to <out>: ncol nsteps out_every pinned
! ms_per_run ms_per_fill column_steps_per_s bytes_up_per_step bytes_down_per_step
! chunks ldasin.
!
! usage: engine_drop_in <run|runl|sflx> <tbl_dir> <in.bin> <out.bin>
!        engine_drop_in time <tbl_dir> <in.bin> <out.txt> <ncol> <nsteps> <out_every> <pinned>
!                            [<chunks>]   (noahmp_run's pipeline chunks, default the module's)
!                            [<ldasin>]   (1: upload the LDASIN block, nmp_ldasin_forcing;
!                                          2: and only its COSZ row on 3 steps of 4)
!   in.bin : int32 n, nsteps, yearlen, options(12); real zsoil(4), dt;
!            real julian(nsteps); int32 static_i(n,6), isnow(n);
!            real static_f(n,6), state(n,56), forcing(n,12,nsteps)
!   out.bin: per step: real state(n,56), int32 isnow(n), real diag(n,58),
!            int32 status(n)
program engine_drop_in
  use iso_c_binding
  use noahmp_global, only: noahmp_set_options
  use noahmp_engine
  implicit none
  character(len=512) :: mode, tbl, fin, fout
  integer :: u, v, n, nsteps, yl, opts(12), s, c
  real :: zs(4), dt
  real, allocatable :: jul(:), sf(:,:), st(:,:), frc(:,:,:)
  integer, allocatable :: si(:,:), isn(:)
  ! LDASIN field f (NMP_L_* + 1) = forcing field lmap(f) (NMP_A_* + 1)
  integer, parameter :: lmap(9) = [1, 6, 4, 5, 3, 9, 7, 8, 10]

  call get_command_argument(1, mode)
  call get_command_argument(2, tbl)
  call get_command_argument(3, fin)
  call get_command_argument(4, fout)
  open(newunit=u, file=trim(fin), access='stream', form='unformatted', status='old')
  read(u) n, nsteps, yl, opts, zs, dt
  allocate(jul(nsteps), si(n, 6), isn(n), sf(n, 6), st(n, 56), frc(n, 12, nsteps))
  read(u) jul, si, isn, sf, st, frc
  close(u)

  call noahmp_set_options(opts(1), opts(2), opts(3), opts(4), opts(5), opts(6), &
                          opts(7), opts(8), opts(9), opts(10), opts(11), opts(12))
  nmp_tbl_dir = tbl
  if (trim(mode) == 'time') then
     call time_run()
     stop
  end if
  call noahmp_columns(n)
  nmp_static_i = si; nmp_isnow = isn; nmp_static_f = sf; nmp_state = st
  nmp_zsoil = zs; nmp_dt = dt; nmp_yearlen = yl; nmp_diag_level = 2
  call noahmp_init()

  open(newunit=v, file=trim(fout), access='stream', form='unformatted', status='replace')
  do s = 1, nsteps
     nmp_julian = jul(s)
     if (trim(mode) == 'run' .or. trim(mode) == 'runl' .or. trim(mode) == 'runc') then
        nmp_ldasin_forcing = trim(mode) /= 'run'
        nmp_ldasin_cosz_only = trim(mode) == 'runc' .and. mod(s - 1, 4) /= 0
        if (nmp_ldasin_forcing) then
           nmp_ldasin = frc(:, lmap, s)
        else
           nmp_forcing = frc(:, :, s)
        end if
        call noahmp_run()
        call noahmp_get_state()
     else
        nmp_status = 0
        do c = 1, n
           call sflx_one(c, s)
        end do
     end if
     write(v) nmp_state, nmp_isnow, nmp_diag, nmp_status
  end do
  close(v)
  call noahmp_finalize()

contains

  subroutine time_run()   ! mode "time": noahmp_run at a production column count
    character(len=64) :: arg
    integer :: ncol, nt, oe, pinned, nf, k, i, j, ldasin
    integer(8) :: t0, t1, t2, rate, trun, tfill
    real, allocatable :: frep(:,:,:), lrep(:,:,:)
    real(8) :: ms_run, ms_fill, up, down
    call get_command_argument(5, arg); read(arg, *) ncol
    call get_command_argument(6, arg); read(arg, *) nt
    call get_command_argument(7, arg); read(arg, *) oe
    call get_command_argument(8, arg); read(arg, *) pinned
    if (command_argument_count() >= 9) then
       call get_command_argument(9, arg); read(arg, *) nmp_chunks
    end if
    ldasin = 0
    if (command_argument_count() >= 10) then
       call get_command_argument(10, arg); read(arg, *) ldasin
    end if
    nmp_ldasin_forcing = ldasin /= 0
    ! (ldasin 2: the timed steps cycle the nf forcing slices; each slice's
    ! LDASIN variables are taken to hold for 4 steps, of which 3 upload COSZ only)
    nf = min(nsteps, 4)
    call noahmp_columns(ncol)
    do i = 1, ncol
       j = mod(i - 1, n) + 1
       nmp_static_i(i, :) = si(j, :); nmp_isnow(i) = isn(j)
       nmp_static_f(i, :) = sf(j, :); nmp_state(i, :) = st(j, :)
    end do
    allocate(frep(ncol, 12, nf), lrep(ncol, 9, nf))
    do k = 1, nf
       do i = 1, ncol
          frep(i, :, k) = frc(mod(i - 1, n) + 1, :, k)
       end do
       lrep(:, :, k) = frep(:, lmap, k)
    end do
    nmp_zsoil = zs; nmp_dt = dt; nmp_yearlen = yl
    nmp_pinned = pinned /= 0
    call noahmp_init()
    trun = 0; tfill = 0
    call system_clock(count_rate=rate)
    up = 0; down = 0
    do s = 1, nt + 2
       k = mod(s - 1, nf) + 1
       call system_clock(t0)
       nmp_ldasin_cosz_only = ldasin == 2 .and. mod(s - 1, 4) /= 0
       if (nmp_ldasin_cosz_only) then       ! the host's own work: filling this step's forcing
          nmp_ldasin(:, 9) = lrep(:, 9, k)
       else if (nmp_ldasin_forcing) then
          nmp_ldasin = lrep(:, :, k)
       else
          nmp_forcing = frep(:, :, k)
       end if
       nmp_julian = jul(k)
       nmp_diag_level = merge(1, 0, mod(s, oe) == 0)
       call system_clock(t1)
       call noahmp_run()
       call system_clock(t2)
       if (s > 2) then
          tfill = tfill + (t1 - t0); trun = trun + (t2 - t1)
          up = up + merge(4d0 * merge(1, 9, nmp_ldasin_cosz_only), &
                          storage_size(nmp_forcing) / 8d0 * 12, nmp_ldasin_forcing) * ncol
          down = down + ncol * (4d0 + storage_size(nmp_diag) / 8d0 * merge(16, 0, nmp_diag_level == 1))
       end if
    end do
    call noahmp_get_state()
    ms_run = 1d3 * real(trun, 8) / real(rate, 8) / nt
    ms_fill = 1d3 * real(tfill, 8) / real(rate, 8) / nt
    open(newunit=v, file=trim(fout), status='replace')
    write(v, '(i0, 1x, i0, 1x, i0, 1x, i0, 1x, es14.6, 1x, es14.6, 1x, es14.6, 1x, es14.6, 1x, es14.6, &
         & 1x, i0, 1x, i0)') ncol, nt, oe, pinned, ms_run, ms_fill, ncol / (ms_run * 1d-3), up / nt, &
         down / nt, nmp_chunks, ldasin
    close(v)
    call noahmp_finalize()
  end subroutine

  subroutine sflx_one(c, s)   ! column c, step s: the reference's calling sequence
    integer, intent(in) :: c, s
    real :: ficeold(-2:0), stc(-2:4), zsnso(-2:4), snice(-2:0), snliq(-2:0), sw(4), smc(4)
    real :: zlvl, o(58), stl(56)
    integer :: isnow, iz
    stl = real(nmp_state(c, :))   ! the reference's default real (nmp_rk may be c_double)
    stc = stl(1:7); zsnso = stl(8:14)
    snice = stl(15:17); snliq = stl(18:20)
    sw = stl(21:24); smc = stl(25:28)
    isnow = nmp_isnow(c)
    ficeold = 0.0
    do iz = isnow + 1, 0
       ficeold(iz) = snice(iz) / (snice(iz) + snliq(iz))
    end do
    zlvl = real(nmp_static_f(c, 2))
    o = 0.0
    call noahmp_sflx(c, 1, real(nmp_static_f(c, 1)), yl, jul(s), frc(c, 10, s), &
         dt, 1000.0, 20.0, 4, nmp_zsoil, 3, &
         real(nmp_static_f(c, 3)), real(nmp_static_f(c, 4)), nmp_static_i(c, 3), nmp_static_i(c, 2), &
         nmp_static_i(c, 1), nmp_static_i(c, 6), nmp_static_i(c, 5), &
         nmp_static_i(c, 4), &
         0, &
         frc(c, 1, s), frc(c, 2, s), frc(c, 3, s), frc(c, 4, s), frc(c, 5, s), frc(c, 6, s), &
         0.0, frc(c, 7, s), frc(c, 8, s), frc(c, 9, s), real(nmp_static_f(c, 5)), frc(c, 11, s), &
         frc(c, 12, s), real(nmp_static_f(c, 6)), ficeold, 1000.0, zlvl, &
         stl(40), stl(39), &
         stc, sw, smc, stl(31), stl(32), stl(33), &
         stl(34), stl(35), stl(29), stl(30), &
         stl(36), stl(42), &
         isnow, zsnso, stl(37), stl(38), snice, snliq, &
         stl(43), stl(44), stl(45), stl(46), &
         stl(49), stl(50), &
         stl(51), stl(52), stl(53), stl(54), &
         stl(47), stl(48), &
         stl(55), stl(56), stl(41), &
         o(1), o(2), o(3), o(4), o(5), o(6), o(7), o(8), o(9), o(10), o(11), o(12), &
         o(13), o(14), o(15), o(16), o(17), o(18), o(19), o(20), o(21), o(22), o(23), o(24), &
         o(25), o(26), o(27), o(28), o(29), o(30), o(31), o(32), o(33), o(34), o(35), o(36), &
         o(37), o(38), o(39), o(40), o(41), o(42), o(43), o(44), o(45), o(46), o(47), o(48), &
         o(49), o(50), o(51), o(52), o(53), o(54), o(55), o(56), o(57), o(58))
    stl(1:7) = stc; stl(8:14) = zsnso; stl(15:17) = snice; stl(18:20) = snliq
    stl(21:24) = sw; stl(25:28) = smc
    nmp_state(c, :) = stl
    nmp_isnow(c) = isnow
    nmp_diag(c, :) = o
    nmp_status(c) = nmp_sflx_status
  end subroutine

end program
