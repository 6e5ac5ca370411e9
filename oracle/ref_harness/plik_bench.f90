! ORACLE TEST INFRASTRUCTURE -- CPU baseline timing of the REFERENCE's own
! TPlikLiteLikelihood_LogLike (source/CMB.f90:305-329, compiled from
! /root/reference by oracle/Makefile).  Used only by bench.py's cpu_baseline.
!
! usage: plik_bench <likelihoods.ini> <theory.bin> <nuis.bin> <W> <lmax> <nfield> <n_nuis> <seconds>
!   loads W walkers once, then evaluates LogLike cycling over them for about
!   <seconds> of wall time (checked every 64 evaluations); prints
!   "<evals> <seconds> <sum of -lnL>"
program plik_bench
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
    Type(TCosmoTheoryPredictions), allocatable :: Th(:)
    Type(CMBParams) :: CMB
    character(LEN=1024) :: ini_name, th_name, nu_name, arg
    integer :: W, lmax, nfield, n_nuis, w_i, f, u_th, u_nu, k
    integer(8) :: c0, c1, rate, nev
    real(mcp), allocatable :: cl(:,:), nuis(:,:)
    real(mcp) :: secs, el, tot
    logical :: bad
    integer, parameter :: fi(10) = [1,2,2,3,3,3,4,4,4,4], fj(10) = [1,1,2,1,2,3,1,2,3,4]

    call get_command_argument(1, ini_name)
    call get_command_argument(2, th_name)
    call get_command_argument(3, nu_name)
    call get_command_argument(4, arg); read(arg, *) W
    call get_command_argument(5, arg); read(arg, *) lmax
    call get_command_argument(6, arg); read(arg, *) nfield
    call get_command_argument(7, arg); read(arg, *) n_nuis
    call get_command_argument(8, arg); read(arg, *) secs
    Feedback = 0
    call Ini%Open(trim(ini_name), bad, .false.)
    if (bad) stop 'cannot open ini'
    call CMBLikelihood_Add(Likes, Ini)
    allocate(Th(W), cl(0:lmax, nfield), nuis(max(n_nuis,1), W))
    open(newunit=u_th, file=trim(th_name), access='stream', form='unformatted', status='old')
    open(newunit=u_nu, file=trim(nu_name), access='stream', form='unformatted', status='old')
    do w_i = 1, W
        read(u_th) cl
        if (n_nuis > 0) read(u_nu) nuis(1:n_nuis, w_i)
        allocate(Th(w_i)%Cls(4,4))
        do f = 1, nfield
            allocate(Th(w_i)%Cls(fi(f), fj(f))%CL(1:lmax))
            Th(w_i)%Cls(fi(f), fj(f))%CL(1:lmax) = cl(1:lmax, f)
        end do
    end do
    close(u_th); close(u_nu)
    tot = 0
    nev = 0
    call system_clock(c0, rate)
    do
        do w_i = 1, 64
            ! one evaluation = every registered likelihood at this point (all
            ! share the same nuisance vector here: calPlanck)
            do k = 1, Likes%Count
                DL => Likes%Item(k)
                select type (DL)
                class is (TCMBLikelihood)
                    tot = tot + DL%LogLike(CMB, Th(mod(nev, int(W,8)) + 1), nuis(:, mod(nev, int(W,8)) + 1))
                end select
            end do
            nev = nev + 1
        end do
        call system_clock(c1)
        el = real(c1 - c0, mcp) / real(rate, mcp)
        if (el >= secs) exit
    end do
    write(*, '(I12, 2ES25.16)') nev, el, tot
end program plik_bench
