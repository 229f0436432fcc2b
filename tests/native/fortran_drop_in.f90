! The Fortran drop-in of INTEGRATION.md, exercised at run time: the module
! `noahmp_func_mi355x` (extracted verbatim from INTEGRATION.md by
! __graft_entry__.build()) replaces the reference's public frh2o and calhum
! (core/module_noahmp_func.f90:4494, :3958) with the engine's C ABI, and this
! program calls them exactly as reference code would -- one scalar call per
! column -- for the inputs in a stream file.  tests/test_gpu_routines.py
! compares the outputs with the reference routines themselves.
!
! usage: fortran_drop_in <tbl_dir> <in.bin> <out.bin>
!   in.bin : int32 n, then int32 sltyp(n), real tkelv(n), smc(n), sh2o(n),
!            sfctmp(n), sfcprs(n)
!   out.bin: real free(n), real q2sat(n), real dqsdt2(n)
program fortran_drop_in
  use iso_c_binding
  use noahmp_func_mi355x
  implicit none
  interface
     integer(c_int) function nmp_read_tables(dir, soil, veg, params) bind(C)
       import; character(kind=c_char) :: dir(*), soil(*), veg(*); type(c_ptr), value :: params
     end function
     integer(c_int) function nmp_init(params, opts, device, precision, eng) bind(C)
       import; type(c_ptr), value :: params, opts
       integer(c_int), value :: device, precision; type(c_ptr) :: eng
     end function
  end interface
  integer(c_int8_t), allocatable, target :: params(:)
  integer(c_int32_t), target :: opts(12)
  character(len=512) :: tbl, fin, fout
  integer :: u, n, i, rc
  integer(c_int32_t), allocatable :: sltyp(:)
  real, allocatable :: tk(:), smc(:), sh2o(:), t(:), p(:), fr(:), q(:), d(:)

  call get_command_argument(1, tbl)
  call get_command_argument(2, fin)
  call get_command_argument(3, fout)
  allocate(params(65536))   ! >= sizeof(nmp_params)
  rc = nmp_read_tables(trim(tbl)//c_null_char, "STAS"//c_null_char, "USGS"//c_null_char, &
                       c_loc(params))
  if (rc /= 0) stop 'nmp_read_tables'
  opts = [1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1]   ! run/case.nml's options
  rc = nmp_init(c_loc(params), c_loc(opts), 0_c_int, 4_c_int, nmp_eng)
  if (rc /= 0) stop 'nmp_init'

  open(newunit=u, file=trim(fin), access='stream', form='unformatted', status='old')
  read(u) n
  allocate(sltyp(n), tk(n), smc(n), sh2o(n), t(n), p(n), fr(n), q(n), d(n))
  read(u) sltyp, tk, smc, sh2o, t, p
  close(u)
  do i = 1, n   ! the reference's calling pattern: scalar calls
     call frh2o(sltyp(i), fr(i), tk(i), smc(i), sh2o(i))
     call calhum(t(i), p(i), q(i), d(i))
  end do
  open(newunit=u, file=trim(fout), access='stream', form='unformatted', status='replace')
  write(u) fr, q, d
  close(u)
end program
