! ORACLE TEST INFRASTRUCTURE -- never shipped, never part of the product path.
!
! The Fortran side of the drop-in (INTEGRATION.md section 2): the NativeCMB
! module extracted from INTEGRATION.md, compiled against the reference's own
! modules, evaluated like plik_harness evaluates the reference's likelihoods
! (Theory%Cls from a stream file, LogLike(CMB, Theory, DataParams) per walker)
! but through TNativeCMBLike, i.e. libcosmomc_amd's cmbl_loglike_batch_host.
!
! usage: native_check <tag> <dataset> <theory.bin> <nuis.bin> <W> <lmax> <nfield> <n_nuis> <out.txt>
program native_check
    use settings
    use CosmologyTypes
    use CosmoTheory
    use NativeCMB
    implicit none
    class(TNativeCMBLike), pointer :: like
    Type(TCosmoTheoryPredictions) :: Theory
    Type(CMBParams) :: CMB
    character(LEN=1024) :: tag, ds, th_name, nu_name, out_name, arg
    integer :: W, lmax, nfield, n_nuis, w_i, f, u_th, u_nu, u_out
    real(mcp), allocatable :: cl(:,:), nuis(:)
    integer, parameter :: fi(10) = [1,2,2,3,3,3,4,4,4,4], fj(10) = [1,1,2,1,2,3,1,2,3,4]

    call get_command_argument(1, tag)
    call get_command_argument(2, ds)
    call get_command_argument(3, th_name)
    call get_command_argument(4, nu_name)
    call get_command_argument(5, arg); read(arg, *) W
    call get_command_argument(6, arg); read(arg, *) lmax
    call get_command_argument(7, arg); read(arg, *) nfield
    call get_command_argument(8, arg); read(arg, *) n_nuis
    call get_command_argument(9, out_name)
    Feedback = 0
    like => NativeCMB_Open(trim(tag), trim(ds), '')
    allocate(Theory%Cls(4,4))
    do f = 1, nfield
        allocate(Theory%Cls(fi(f), fj(f))%CL(1:lmax))
    end do
    allocate(cl(0:lmax, nfield), nuis(n_nuis))
    open(newunit=u_th, file=trim(th_name), access='stream', form='unformatted', status='old')
    open(newunit=u_nu, file=trim(nu_name), access='stream', form='unformatted', status='old')
    open(newunit=u_out, file=trim(out_name), status='replace')
    do w_i = 1, W
        read(u_th) cl
        if (n_nuis > 0) read(u_nu) nuis
        do f = 1, nfield
            Theory%Cls(fi(f), fj(f))%CL(1:lmax) = cl(1:lmax, f)
        end do
        write(u_out, '(ES25.17)') like%LogLike(CMB, Theory, nuis)
    end do
    close(u_th); close(u_nu); close(u_out)
end program native_check
