! Fortran 2003 bindings (iso_c_binding) for the C API (reference capability:
! the generated Fortran module of tools/fortran/generate_fortran_module.py).
! Only handles, creation from LAPACK arrays and the simplified-API drivers
! are bound; scalars are passed by value as in c_api.h.
module slate_amd
    use iso_c_binding
    implicit none

    type, bind(c) :: slate_Options
        integer(c_int) :: option
        integer(c_int64_t) :: ivalue
        real(c_double) :: dvalue
    end type slate_Options

    interface
        function slate_version() bind(c, name="slate_version")
            import :: c_ptr
            type(c_ptr) :: slate_version
        end function

        ! process grid over a torchrun-style launch (RANK / WORLD_SIZE env)
        function slate_grid_init(p, q) bind(c, name="slate_grid_init")
            import :: c_int
            integer(c_int), value :: p, q
            integer(c_int) :: slate_grid_init
        end function

        function slate_grid_rank() bind(c, name="slate_grid_rank")
            import :: c_int
            integer(c_int) :: slate_grid_rank
        end function

        function slate_grid_size() bind(c, name="slate_grid_size")
            import :: c_int
            integer(c_int) :: slate_grid_size
        end function

        subroutine slate_finalize() bind(c, name="slate_finalize")
        end subroutine

        function slate_Matrix_create_fromLAPACK_r64(m, n, A, lda, nb) &
                bind(c, name="slate_Matrix_create_fromLAPACK_r64")
            import :: c_ptr, c_int64_t, c_double
            integer(c_int64_t), value :: m, n, lda, nb
            real(c_double) :: A(lda, *)
            type(c_ptr) :: slate_Matrix_create_fromLAPACK_r64
        end function

        function slate_Matrix_create_fromLAPACK_c64(m, n, A, lda, nb) &
                bind(c, name="slate_Matrix_create_fromLAPACK_c64")
            import :: c_ptr, c_int64_t, c_double_complex
            integer(c_int64_t), value :: m, n, lda, nb
            complex(c_double_complex) :: A(lda, *)
            type(c_ptr) :: slate_Matrix_create_fromLAPACK_c64
        end function

        subroutine slate_Matrix_destroy_r64(A) bind(c, name="slate_Matrix_destroy_r64")
            import :: c_ptr
            type(c_ptr), value :: A
        end subroutine

        subroutine slate_Matrix_destroy_c64(A) bind(c, name="slate_Matrix_destroy_c64")
            import :: c_ptr
            type(c_ptr), value :: A
        end subroutine

        subroutine slate_Matrix_tileUpdateAllOrigin_r64(A) bind(c, name="slate_Matrix_tileUpdateAllOrigin_r64")
            import :: c_ptr
            type(c_ptr), value :: A
        end subroutine

        function slate_multiply_r64(alpha, A, B, beta, C, nopts, opts) bind(c, name="slate_multiply_r64")
            import :: c_ptr, c_int, c_double, slate_Options
            real(c_double), value :: alpha, beta
            type(c_ptr), value :: A, B, C
            integer(c_int), value :: nopts
            type(slate_Options) :: opts(*)
            integer(c_int) :: slate_multiply_r64
        end function

        function slate_lu_solve_r64(A, B, nopts, opts) bind(c, name="slate_lu_solve_r64")
            import :: c_ptr, c_int, c_int64_t, slate_Options
            type(c_ptr), value :: A, B
            integer(c_int), value :: nopts
            type(slate_Options) :: opts(*)
            integer(c_int64_t) :: slate_lu_solve_r64
        end function

        function slate_chol_solve_r64(uplo, A, B, nopts, opts) bind(c, name="slate_chol_solve_r64")
            import :: c_ptr, c_int, c_int64_t, c_char, slate_Options
            character(kind=c_char), value :: uplo
            type(c_ptr), value :: A, B
            integer(c_int), value :: nopts
            type(slate_Options) :: opts(*)
            integer(c_int64_t) :: slate_chol_solve_r64
        end function

        function slate_least_squares_solve_r64(A, BX, nopts, opts) bind(c, name="slate_least_squares_solve_r64")
            import :: c_ptr, c_int, slate_Options
            type(c_ptr), value :: A, BX
            integer(c_int), value :: nopts
            type(slate_Options) :: opts(*)
            integer(c_int) :: slate_least_squares_solve_r64
        end function

        function slate_hermitian_eig_r64(uplo, A, Lambda, Z, nopts, opts) bind(c, name="slate_hermitian_eig_r64")
            import :: c_ptr, c_int, c_char, c_double, slate_Options
            character(kind=c_char), value :: uplo
            type(c_ptr), value :: A, Z
            real(c_double) :: Lambda(*)
            integer(c_int), value :: nopts
            type(slate_Options) :: opts(*)
            integer(c_int) :: slate_hermitian_eig_r64
        end function

        function slate_svd_r64(A, Sigma, U, VT, nopts, opts) bind(c, name="slate_svd_r64")
            import :: c_ptr, c_int, c_double, slate_Options
            type(c_ptr), value :: A, U, VT
            real(c_double) :: Sigma(*)
            integer(c_int), value :: nopts
            type(slate_Options) :: opts(*)
            integer(c_int) :: slate_svd_r64
        end function
    end interface
end module slate_amd
