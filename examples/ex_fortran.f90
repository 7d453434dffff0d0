! Fortran example through the slate_amd module (host target): LU solve,
! Cholesky factor + solve-using-factor, one-norm, complex GEMM, QR least
! squares and a generated test matrix.  Stops with a nonzero code on error.
program ex_fortran
    use slate_amd
    implicit none
    integer(c_int64_t), parameter :: n = 200, nb = 64, m = 260
    real(c_double) :: A(n, n), A0(n, n), B(n, 1), B0(n, 1), S(n, n), X(n, 1)
    real(c_double) :: L(m, n), L0(m, n), R(m, 1), R0(m, 1), G(n, n)
    complex(c_double_complex) :: Ca(n, n), Cb(n, n), Cc(n, n)
    real(c_double) :: re(n, n), im(n, n)
    type(c_ptr) :: As, Bs, Ss, Xs, Ls, Rs, Gs, Cas, Cbs, Ccs
    type(slate_Options) :: opts(1)
    integer(c_int64_t) :: info
    real(c_double) :: nrm, err
    integer :: i, rc
    opts(1) = slate_Options(slate_Option_Target, ichar('H'), 0d0)

    ! LU solve
    call random_number(A)
    do i = 1, int(n)
        A(i, i) = A(i, i) + n
    end do
    call random_number(B)
    A0 = A
    B0 = B
    As = slate_Matrix_create_fromLAPACK_r64(n, n, A, n, nb)
    Bs = slate_Matrix_create_fromLAPACK_r64(n, 1_c_int64_t, B, n, nb)
    info = slate_lu_solve_r64(As, Bs, 1, opts)
    call slate_Matrix_tileUpdateAllOrigin_r64(Bs)
    err = maxval(abs(matmul(A0, B) - B0))
    print '(a, i0, a, es10.3)', 'lu_solve info = ', info, '  max|Ax-b| = ', err
    if (info /= 0 .or. err > 1d-10) stop 1
    call slate_Matrix_destroy_r64(As)
    call slate_Matrix_destroy_r64(Bs)

    ! one-norm of A0 against Fortran
    As = slate_Matrix_create_fromLAPACK_r64(n, n, A0, n, nb)
    nrm = slate_norm_r64('1', As, 1, opts)
    print '(a, es12.5)', 'norm1 rel err = ', abs(nrm - maxval(sum(abs(A0), 1))) / nrm
    if (abs(nrm - maxval(sum(abs(A0), 1))) > 1d-12 * nrm) stop 2
    call slate_Matrix_destroy_r64(As)

    ! Cholesky factor, then solve using the factor (lower triangle)
    S = matmul(transpose(A0), A0)
    Ss = slate_Matrix_create_fromLAPACK_r64(n, n, S, n, nb)
    info = slate_chol_factor_r64('L', Ss, 1, opts)
    X = B0
    Xs = slate_Matrix_create_fromLAPACK_r64(n, 1_c_int64_t, X, n, nb)
    rc = slate_chol_solve_using_factor_r64('L', Ss, Xs, 1, opts)
    call slate_Matrix_tileUpdateAllOrigin_r64(Xs)
    err = maxval(abs(matmul(matmul(transpose(A0), A0), X) - B0)) / maxval(abs(B0))
    print '(a, i0, a, es10.3)', 'chol info = ', info, '  rel resid = ', err
    if (info /= 0 .or. rc /= 0 .or. err > 1d-8) stop 3
    call slate_Matrix_destroy_r64(Ss)
    call slate_Matrix_destroy_r64(Xs)

    ! complex GEMM C = A B
    call random_number(re)
    call random_number(im)
    Ca = cmplx(re, im, kind=c_double_complex)
    call random_number(re)
    call random_number(im)
    Cb = cmplx(re, im, kind=c_double_complex)
    Cc = (0d0, 0d0)
    Cas = slate_Matrix_create_fromLAPACK_c64(n, n, Ca, n, nb)
    Cbs = slate_Matrix_create_fromLAPACK_c64(n, n, Cb, n, nb)
    Ccs = slate_Matrix_create_fromLAPACK_c64(n, n, Cc, n, nb)
    rc = slate_multiply_c64((1d0, 0d0), Cas, Cbs, (0d0, 0d0), Ccs, 1, opts)
    call slate_Matrix_tileUpdateAllOrigin_c64(Ccs)
    err = maxval(abs(Cc - matmul(Ca, Cb)))
    print '(a, es10.3)', 'zgemm max err = ', err
    if (rc /= 0 .or. err > 1d-10) stop 4
    call slate_Matrix_destroy_c64(Cas)
    call slate_Matrix_destroy_c64(Cbs)
    call slate_Matrix_destroy_c64(Ccs)

    ! least squares min |L x - r| (m > n): the normal equations hold at the solution
    call random_number(L)
    call random_number(R)
    R0 = R
    L0 = L
    G = 0
    Ls = slate_Matrix_create_fromLAPACK_r64(m, n, L, m, nb)
    Rs = slate_Matrix_create_fromLAPACK_r64(m, 1_c_int64_t, R, m, nb)
    rc = slate_least_squares_solve_r64(Ls, Rs, 1, opts)
    call slate_Matrix_tileUpdateAllOrigin_r64(Rs)
    err = maxval(abs(matmul(transpose(L0), matmul(L0, R(1:n, :)) - R0))) / maxval(abs(matmul(transpose(L0), R0)))
    print '(a, i0, a, es10.3)', 'gels rc = ', rc, '  normal-eq resid = ', err
    if (rc /= 0 .or. err > 1d-10) stop 6
    call slate_Matrix_destroy_r64(Ls)
    call slate_Matrix_destroy_r64(Rs)

    ! generated matrix: 'spd' is symmetric positive definite
    Gs = slate_Matrix_create_fromLAPACK_r64(n, n, G, n, nb)
    rc = slate_generate_matrix_r64('spd'//c_null_char, Gs, 7_c_int64_t, -1d0, 1, opts)
    call slate_Matrix_tileUpdateAllOrigin_r64(Gs)
    info = slate_chol_factor_r64('L', Gs, 1, opts)
    print '(a, i0, a, i0)', 'generate spd rc = ', rc, '  potrf info = ', info
    if (rc /= 0 .or. info /= 0) stop 5
    call slate_Matrix_destroy_r64(Gs)
end program ex_fortran
