! The Fortran engine slot of INTEGRATION.md, exercised at run time.  The module
! `noahmp_engine` (extracted verbatim from INTEGRATION.md by
! __graft_entry__.build()) replaces the reference's empty engine slot
! (core/module_noahmp_engine.f90:5-10).  This program drives it the way a
! Fortran host of the reference would: options through the reference's own
! noahmp_set_options (module noahmp_global, compiled from /root/reference by
! oracle/Makefile), then either
!   mode "run" : noahmp_init once, noahmp_run every step over the module's
!                column arrays (state resident on the device), or
!   mode "sflx": one noahmp_sflx call per column per step with the
!                reference's 131 arguments (FICEOLD from the step-start ice
!                fraction, as the reference harness passes it).
! tests/test_gpu_routines.py compares every step with the reference trajectory.
!
! usage: engine_drop_in <run|sflx> <tbl_dir> <in.bin> <out.bin>
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
  call noahmp_columns(n)
  nmp_static_i = si; nmp_isnow = isn; nmp_static_f = sf; nmp_state = st
  nmp_zsoil = zs; nmp_dt = dt; nmp_yearlen = yl; nmp_diag_level = 2
  call noahmp_init()

  open(newunit=v, file=trim(fout), access='stream', form='unformatted', status='replace')
  do s = 1, nsteps
     nmp_julian = jul(s)
     if (trim(mode) == 'run') then
        nmp_forcing = frc(:, :, s)
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

  subroutine sflx_one(c, s)   ! column c, step s: the reference's calling sequence
    integer, intent(in) :: c, s
    real :: ficeold(-2:0), stc(-2:4), zsnso(-2:4), snice(-2:0), snliq(-2:0), sw(4), smc(4)
    real :: zlvl, o(58)
    integer :: isnow, iz
    stc = nmp_state(c, 1:7); zsnso = nmp_state(c, 8:14)
    snice = nmp_state(c, 15:17); snliq = nmp_state(c, 18:20)
    sw = nmp_state(c, 21:24); smc = nmp_state(c, 25:28)
    isnow = nmp_isnow(c)
    ficeold = 0.0
    do iz = isnow + 1, 0
       ficeold(iz) = snice(iz) / (snice(iz) + snliq(iz))
    end do
    zlvl = nmp_static_f(c, 2)
    o = 0.0
    call noahmp_sflx(c, 1, nmp_static_f(c, 1), yl, jul(s), frc(c, 10, s), &
         dt, 1000.0, 20.0, 4, nmp_zsoil, 3, &
         nmp_static_f(c, 3), nmp_static_f(c, 4), nmp_static_i(c, 3), nmp_static_i(c, 2), &
         nmp_static_i(c, 1), nmp_static_i(c, 6), nmp_static_i(c, 5), &
         nmp_static_i(c, 4), &
         0, &
         frc(c, 1, s), frc(c, 2, s), frc(c, 3, s), frc(c, 4, s), frc(c, 5, s), frc(c, 6, s), &
         0.0, frc(c, 7, s), frc(c, 8, s), frc(c, 9, s), nmp_static_f(c, 5), frc(c, 11, s), &
         frc(c, 12, s), nmp_static_f(c, 6), ficeold, 1000.0, zlvl, &
         nmp_state(c, 40), nmp_state(c, 39), &
         stc, sw, smc, nmp_state(c, 31), nmp_state(c, 32), nmp_state(c, 33), &
         nmp_state(c, 34), nmp_state(c, 35), nmp_state(c, 29), nmp_state(c, 30), &
         nmp_state(c, 36), nmp_state(c, 42), &
         isnow, zsnso, nmp_state(c, 37), nmp_state(c, 38), snice, snliq, &
         nmp_state(c, 43), nmp_state(c, 44), nmp_state(c, 45), nmp_state(c, 46), &
         nmp_state(c, 49), nmp_state(c, 50), &
         nmp_state(c, 51), nmp_state(c, 52), nmp_state(c, 53), nmp_state(c, 54), &
         nmp_state(c, 47), nmp_state(c, 48), &
         nmp_state(c, 55), nmp_state(c, 56), nmp_state(c, 41), &
         o(1), o(2), o(3), o(4), o(5), o(6), o(7), o(8), o(9), o(10), o(11), o(12), &
         o(13), o(14), o(15), o(16), o(17), o(18), o(19), o(20), o(21), o(22), o(23), o(24), &
         o(25), o(26), o(27), o(28), o(29), o(30), o(31), o(32), o(33), o(34), o(35), o(36), &
         o(37), o(38), o(39), o(40), o(41), o(42), o(43), o(44), o(45), o(46), o(47), o(48), &
         o(49), o(50), o(51), o(52), o(53), o(54), o(55), o(56), o(57), o(58))
    nmp_state(c, 1:7) = stc; nmp_state(c, 8:14) = zsnso
    nmp_state(c, 15:17) = snice; nmp_state(c, 18:20) = snliq
    nmp_state(c, 21:24) = sw; nmp_state(c, 25:28) = smc
    nmp_isnow(c) = isnow
    nmp_diag(c, :) = o
    nmp_status(c) = nmp_sflx_status
  end subroutine

end program
