! ORACLE TEST INFRASTRUCTURE -- never shipped, never part of the product path.
!
! Driver program (written for this repo) that exercises the REFERENCE's own
! compiled RandUtils (source/RandUtils.f90), propose (source/propose.f90) and
! MatrixUtils (source/Matrix_utils_new.f90) modules to produce golden streams:
!
!   mode "kat"    : RANMAR known-answer test (RandUtils.f90:262-283)
!   mode "stream" : ranmar / Gaussian1 / randexp1 / RandIndices / RandRotationD
!   mode "gr"     : GelmanRubinEvalues (samples.f90:41-67) on a given
!                   (mean-of-covariances, covariance-of-means) pair
!   mode "chain"  : (fast_only = 2: TFastDraggingSampler_GetNewSample,
!                   MCMC.f90:338-452, restated inline on the reference's
!                   BlockedProposer GetProposalSlow / GetProposalFastDelta)
!                   BlockedProposer + Metropolis chain on the test_likelihood
!                   Gaussian (calclike.f90:180-199) with hard bounds
!                   (calclike.f90:97-109) and Gaussian priors (:111-134).
!                   The three-line MetropolisAccept of MCMC.f90:119-131 and the
!                   GetLogLike sum (calclike.f90:136-151) are restated inline
!                   (their modules drag in every likelihood); the RNG,
!                   proposer, Cholesky and inverse are the reference's own code.
!
! usage: rng_harness kat|stream|chain|gr <config.txt> <out.txt>
program rng_harness
    use settings
    use RandUtils
    use GeneralTypes
    use MatrixUtils
    use propose
    use Samples, only: GelmanRubinEvalues
    implicit none
    character(LEN=1024) :: mode, cfg, outf
    integer :: u_in, u_out, i, j, k, n, nsteps, nblocks, slow_block_max, oversample, ij, kl, nrot
    integer :: fast_only, nidx
    real(mcp) :: scale, like, curlike, temperature
    real(mcp), allocatable :: cov(:,:), covinv(:,:), P(:), trial(:), center(:), pmin(:), pmax(:)
    real(mcp), allocatable :: pmean(:), pstd(:), R(:,:), X(:)
    integer, allocatable :: bsize(:), ind(:)
    type(int_arr), allocatable :: blocks(:)
    Type(BlockedProposer) :: Prop
    logical :: accpt
    real :: e
    real(mcp), allocatable :: mcov(:,:), evals(:)
    real(mcp), allocatable :: cend(:), cstart(:), tend(:), tstart(:), delta(:)
    real(mcp) :: cendlike, cstartlike, elike, slike, sum_s, sum_e, frac, cintlike, intlike, mult
    integer :: num_drag, num_fast, interp, istep

    call get_command_argument(1, mode)
    call get_command_argument(2, cfg)
    call get_command_argument(3, outf)
    open(newunit=u_out, file=trim(outf), status='replace')
    Rand_Feedback = 0

    select case (trim(mode))
    case ('kat')
        call rmarin(1802, 9373)
        do i = 1, 20000
            like = ranmar()
        end do
        do i = 1, 6
            write(u_out, '(F12.1)') 4096.d0*4096.d0*ranmar()
        end do
    case ('gr')
        open(newunit=u_in, file=trim(cfg), status='old')
        read(u_in, *) n
        allocate(cov(n, n), mcov(n, n), evals(n))
        read(u_in, *) cov
        read(u_in, *) mcov
        close(u_in)
        accpt = GelmanRubinEvalues(cov, mcov, evals, n)
        write(u_out, '(I2)') merge(1, 0, accpt)
        if (accpt) write(u_out, '(ES25.17)') evals
    case ('stream')
        open(newunit=u_in, file=trim(cfg), status='old')
        read(u_in, *) ij, kl, n, nidx, nrot
        close(u_in)
        call initRandom(ij, kl)
        do i = 1, n
            write(u_out, '(ES25.17)') ranmar()
        end do
        do i = 1, n
            write(u_out, '(ES25.17)') Gaussian1()
        end do
        do i = 1, n
            e = randexp1()
            write(u_out, '(ES25.17)') real(e, mcp)
        end do
        allocate(ind(nidx))
        call RandIndices(ind, nidx, nidx)
        do i = 1, nidx
            write(u_out, '(I8)') ind(i)
        end do
        allocate(R(nrot, nrot))
        call RandRotation(R, nrot)
        do i = 1, nrot
            do j = 1, nrot
                write(u_out, '(ES25.17)') R(i, j)
            end do
        end do
    case ('chain')
        open(newunit=u_in, file=trim(cfg), status='old')
        read(u_in, *) ij, kl, n, nsteps, fast_only
        read(u_in, *) nblocks, slow_block_max, oversample, scale, temperature
        allocate(bsize(nblocks), blocks(nblocks))
        read(u_in, *) bsize
        do i = 1, nblocks
            allocate(blocks(i)%P(bsize(i)))
            read(u_in, *) blocks(i)%P
        end do
        allocate(cov(n,n), covinv(n,n), P(n), trial(n), center(n), pmin(n), pmax(n), pmean(n), pstd(n), X(n))
        read(u_in, *) ((cov(i,j), j=1,n), i=1,n)
        read(u_in, *) ((covinv(i,j), j=1,n), i=1,n)
        read(u_in, *) center
        read(u_in, *) pmin
        read(u_in, *) pmax
        read(u_in, *) pmean
        read(u_in, *) pstd
        read(u_in, *) P
        close(u_in)
        num_params = n
        num_params_used = n
        allocate(params_used(n))
        params_used = [(i, i=1,n)]
        call Matrix_Inverse(covinv)          ! test_likelihood inverts its covariance
        call initRandom(ij, kl)
        call Prop%Init(blocks, slow_block_max=slow_block_max, oversample_fast=oversample, &
            propose_scale=scale)
        call Prop%SetCovariance(cov)
        curlike = target(P)
        write(u_out, '(ES25.17)') curlike
        num_fast = 0
        do k = slow_block_max + 1, nblocks
            num_fast = num_fast + bsize(k)
        end do
        allocate(cend(n), cstart(n), tend(n), tstart(n), delta(n))
        num_drag = 0
        mult = 1
        do k = 1, nsteps
            if (fast_only == 2) then
                num_drag = num_drag + 1
                if (mod(num_drag, oversample) == 0) then
                    ! --- TFastDraggingSampler_GetNewSample drag branch (MCMC.f90:364-452)
                    tend = P
                    call Prop%GetProposalSlow(tend)
                    cendlike = target(tend)
                    if (cendlike == LogZero) then
                        mult = mult + 1
                        write(u_out, '(I2,*(ES25.17))') 0, cendlike, curlike, P
                        cycle
                    end if
                    cstartlike = curlike
                    sum_e = cendlike
                    sum_s = cstartlike
                    cstart = P
                    cend = tend
                    interp = max(2, nint(dragging_steps * num_fast) + 1)
                    do istep = 1, interp - 1
                        call Prop%GetProposalFastDelta(delta)
                        tend = cend
                        tend(1:n) = tend(1:n) + delta
                        elike = target(tend)
                        accpt = elike /= LogZero
                        if (accpt) then
                            tstart = cstart
                            tstart(1:n) = tstart(1:n) + delta
                            slike = target(tstart)
                            accpt = slike /= LogZero
                            if (accpt) then
                                frac = real(istep, mcp)/interp
                                cintlike = cstartlike*(1-frac) + frac*cendlike
                                intlike = slike*(1-frac) + frac*elike
                                accpt = cintlike > intlike                 ! MetropolisAccept :119-131
                                if (.not. accpt) accpt = randexp1() > intlike - cintlike
                            end if
                        end if
                        if (accpt) then
                            cend = tend
                            cstart = tstart
                            cendlike = elike
                            cstartlike = slike
                        end if
                        sum_s = sum_s + cstartlike
                        sum_e = sum_e + cendlike
                    end do
                    like = sum_e/interp                     ! DragLike
                    if (like /= LogZero) then
                        accpt = sum_s/interp > like
                        if (.not. accpt) accpt = randexp1() > like - sum_s/interp
                    else
                        accpt = .false.
                    end if
                    if (accpt) then
                        P = cend
                        curlike = cendlike
                        mult = 1
                    else
                        mult = mult + 1
                    end if
                    write(u_out, '(I2,*(ES25.17))') merge(1, 0, accpt), like, curlike, P
                    cycle
                end if
            end if
            trial = P
            if (fast_only >= 1) then
                call Prop%GetProposalFast(trial)
            else
                call Prop%GetProposal(trial)
            end if
            like = target(trial)
            if (like /= LogZero) then               ! MCMC.f90:282-286, :119-131
                accpt = curlike > like
                if (.not. accpt) accpt = randexp1() > like - curlike
            else
                accpt = .false.
            end if
            if (accpt) then
                P = trial
                curlike = like
            end if
            write(u_out, '(I2,*(ES25.17))') merge(1, 0, accpt), like, curlike, P
        end do
    end select
    close(u_out)

contains

    function target(Q) result(L)
        real(mcp), intent(in) :: Q(:)
        real(mcp) :: L, main, pri
        if (any(Q > pmax) .or. any(Q < pmin)) then
            L = LogZero
            return
        end if
        X = Q - center
        main = dot_product(X, matmul(covinv, X))/2
        L = main/temperature
        pri = 0
        do i = 1, n
            if (pstd(i) /= 0) pri = pri + ((Q(i) - pmean(i))/pstd(i))**2
        end do
        L = L + (pri/2)/temperature
    end function target

end program rng_harness
