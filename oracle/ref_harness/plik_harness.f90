! ORACLE TEST INFRASTRUCTURE -- never shipped, never part of the product path.
!
! Driver program (written for this repo) that exercises the REFERENCE's own
! compiled modules, built from /root/reference/source by oracle/Makefile, to
! produce golden -lnL values for the CMB likelihoods on the fast path.
!
! It registers datasets exactly as CosmoMC does, through
! CMBLikelihood_Add (reference source/CMB.f90:54-123), then calls each
! likelihood's LogLike(CMB, Theory, DataParams) (source/CMB.f90:305-329 for
! PLIK_LITE, source/CMBlikes.f90:1165-1227 for CMBLike2 datasets,
! source/CMB_BK_Planck.f90 for BKPLANCK) on theory C_l read from a binary
! stream file.
!
! usage: plik_harness <likelihoods.ini> <theory.bin> <nuis.bin> <W> <lmax> <nfield> <n_nuis> <out.txt> [derived.txt]
!   theory.bin : W x nfield x (lmax+1) float64, field order TT TE EE BT BE BB PT PE PB PP
!                (Theory%Cls(i,j), i>=j, T=1 E=2 B=3 P=4), l = 0..lmax
!   nuis.bin   : W x n_nuis float64 (DataParams of the first likelihood)
!   out.txt    : one -lnL per walker ("%24.17e")
!   derived.txt: (optional) the likelihood's derivedParameters(Theory, DataParams)
!                per walker (GeneralTypes.f90:504-512, CMBlikes.f90:1324-1337 for SMICA)
program plik_harness
    use settings
    use IniObjects
    use GeneralTypes
    use CosmologyTypes
    use CosmoTheory
    use Likelihood_Cosmology
    use CMBLikelihoods
    implicit none
    Type(TSettingIni) :: Ini
    Type(TLikelihoodList), target :: Likes
    class(TDataLikelihood), pointer :: DL
    Type(TCosmoTheoryPredictions) :: Theory
    Type(CMBParams) :: CMB
    character(LEN=1024) :: ini_name, th_name, nu_name, out_name, der_name, arg
    integer :: W, lmax, nfield, n_nuis, w_i, f, i, j, ix, u_th, u_nu, u_out, u_der, nder
    real(mcp), allocatable :: cl(:,:), nuis(:), der(:)
    real(mcp) :: lnl
    logical :: bad
    integer, parameter :: fi(10) = [1,2,2,3,3,3,4,4,4,4], fj(10) = [1,1,2,1,2,3,1,2,3,4]

    call get_command_argument(1, ini_name)
    call get_command_argument(2, th_name)
    call get_command_argument(3, nu_name)
    call get_command_argument(4, arg); read(arg, *) W
    call get_command_argument(5, arg); read(arg, *) lmax
    call get_command_argument(6, arg); read(arg, *) nfield
    call get_command_argument(7, arg); read(arg, *) n_nuis
    call get_command_argument(8, out_name)
    der_name = ''
    if (command_argument_count() >= 9) call get_command_argument(9, der_name)

    Feedback = 0
    call Ini%Open(trim(ini_name), bad, .false.)
    if (bad) stop 'cannot open ini'
    call CMBLikelihood_Add(Likes, Ini)
    if (Likes%Count < 1) stop 'no likelihood registered'

    allocate(Theory%Cls(4,4))
    do f = 1, nfield
        allocate(Theory%Cls(fi(f), fj(f))%CL(1:lmax))
    end do
    allocate(cl(0:lmax, nfield), nuis(n_nuis))

    open(newunit=u_th, file=trim(th_name), access='stream', form='unformatted', status='old')
    open(newunit=u_nu, file=trim(nu_name), access='stream', form='unformatted', status='old')
    open(newunit=u_out, file=trim(out_name), status='replace')
    DL => Likes%Item(1)
    nder = DL%nuisance_params%num_derived
    if (der_name /= '') open(newunit=u_der, file=trim(der_name), status='replace')
    do w_i = 1, W
        read(u_th) cl
        if (n_nuis > 0) read(u_nu) nuis
        do f = 1, nfield
            Theory%Cls(fi(f), fj(f))%CL(1:lmax) = cl(1:lmax, f)
        end do
        select type (DL)
        class is (TCMBLikelihood)
            lnl = DL%LogLike(CMB, Theory, nuis)
        class default
            stop 'not a CMB likelihood'
        end select
        write(u_out, '(ES25.17)') lnl
        if (der_name /= '') then
            if (nder > 0) then
                der = DL%derivedParameters(Theory, nuis)
                write(u_der, '(*(ES25.17))') der
            else
                write(u_der, '(a)') ''
            end if
        end if
    end do
    close(u_th); close(u_nu); close(u_out)
    if (der_name /= '') close(u_der)
    ix = 0; i = 0; j = 0
end program plik_harness
