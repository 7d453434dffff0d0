! Fortran example: LU solve through the slate_amd module (host target).
program ex_fortran
    use slate_amd
    implicit none
    integer(c_int64_t), parameter :: n = 200, nb = 64
    real(c_double) :: A(n, n), A0(n, n), B(n, 1), B0(n, 1)
    type(c_ptr) :: As, Bs
    type(slate_Options) :: opts(1)
    integer(c_int64_t) :: info
    integer :: i
    call random_number(A)
    do i = 1, int(n)
        A(i, i) = A(i, i) + n
    end do
    call random_number(B)
    A0 = A
    B0 = B
    opts(1)%option = 6
    opts(1)%ivalue = ichar('H')
    opts(1)%dvalue = 0d0
    As = slate_Matrix_create_fromLAPACK_r64(n, n, A, n, nb)
    Bs = slate_Matrix_create_fromLAPACK_r64(n, 1_c_int64_t, B, n, nb)
    info = slate_lu_solve_r64(As, Bs, 1, opts)
    call slate_Matrix_tileUpdateAllOrigin_r64(Bs)
    print '(a, i0, a, es10.3)', 'info = ', info, '  max|Ax-b| = ', maxval(abs(matmul(A0, B) - B0))
    call slate_Matrix_destroy_r64(As)
    call slate_Matrix_destroy_r64(Bs)
    if (info /= 0 .or. maxval(abs(matmul(A0, B) - B0)) > 1d-10) stop 1
end program ex_fortran
