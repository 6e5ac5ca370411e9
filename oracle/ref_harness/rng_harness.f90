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
!   mode "confid" : TSampleList%ConfidVal (samples.f90:70-110), the per-chain
!                   limits of CheckLimitsConverge (SampleCollector.f90:515-517)
!   mode "chain"  : (fast_only = 2: TFastDraggingSampler_GetNewSample,
!                   MCMC.f90:338-452, restated inline on the reference's
!                   BlockedProposer GetProposalSlow / GetProposalFastDelta)
!                   BlockedProposer + Metropolis chain on the test_likelihood
!                   Gaussian.  Every -lnL is the reference's own
!                   TLikeCalculator%GetLogLike (calclike.f90:136-151: hard
!                   bounds :97-109, TestLikelihoodFunction :180-199, Gaussian
!                   and linear-combination priors with the
!                   include_fixed_parameter_priors gate :111-134, temperature
!                   :82-94) on BaseParams set from the config; num_params may
!                   exceed num_params_used (fixed parameters).  Only the
!                   three-line MetropolisAccept of MCMC.f90:119-131 is restated
!                   inline; the RNG, proposer, Cholesky and inverse are the
!                   reference's own code.
!   mode "blocks" : TBaseParameters_SetFastSlowParams (BaseParameters.f90:302-433)
!                   on BaseParams%varying and a DataLikelihoods list of plain
!                   TDataLikelihood items carrying new_param_block_start /
!                   new_params / speed, the blocking keys read from the config
!                   itself (an ini file); writes every param_blocks entry
!
! usage: rng_harness kat|stream|chain|gr|confid|blocks <config> <out.txt>
program rng_harness
    use settings
    use StringUtils, only: numcat
    use IniObjects
    use RandUtils
    use GeneralTypes
    use MatrixUtils
    use propose
    use Samples, only: GelmanRubinEvalues, TSampleList
    use BaseParameters
    use CalcLike
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
    integer :: n_used, incl_fixed, nlin, ix1, ix2
    Type(TSampleList) :: SL
    real(mcp) :: limfrac, lower, upper
    Type(TGenericLikeCalculator) :: Calc
    Type(TCalculationAtParamPoint) :: Pt
    Type(TSettingIni) :: BIni
    class(TDataLikelihood), pointer :: BLike
    logical :: bad
    integer, allocatable :: ivec(:)

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
    case ('confid')
        open(newunit=u_in, file=trim(cfg), status='old')
        read(u_in, *) n, nidx, ix1, ix2, limfrac
        allocate(R(nidx, n))
        read(u_in, *) ((R(j, i), j=1,nidx), i=1,n)
        close(u_in)
        do i = 1, n
            call SL%Add(R(:, i))
        end do
        do j = 1, nidx
            call SL%ConfidVal(j, limfrac, ix1, ix2, lower, upper)
            write(u_out, '(2ES25.17)') lower, upper
        end do
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
        read(u_in, *) ij, kl, n, n_used, nsteps, fast_only, incl_fixed, nlin
        read(u_in, *) nblocks, slow_block_max, oversample, scale, temperature
        num_params = n
        num_params_used = n_used
        allocate(params_used(n_used))
        read(u_in, *) params_used
        allocate(bsize(nblocks), blocks(nblocks))
        read(u_in, *) bsize
        do i = 1, nblocks
            allocate(blocks(i)%P(bsize(i)))
            read(u_in, *) blocks(i)%P
        end do
        allocate(cov(n_used,n_used), P(n), trial(n), center(n), pmin(n), pmax(n), pmean(n), pstd(n))
        read(u_in, *) ((cov(i,j), j=1,n_used), i=1,n_used)
        read(u_in, *) center
        read(u_in, *) pmin
        read(u_in, *) pmax
        read(u_in, *) pmean
        read(u_in, *) pstd
        read(u_in, *) P
        ! BaseParams as TBaseParameters_ReadParams / ReadPriors leave them (BaseParameters.f90:60-203)
        allocate(BaseParams%PMin(n), BaseParams%PMax(n), BaseParams%center(n), BaseParams%varying(n))
        allocate(BaseParams%GaussPriors%mean(n), BaseParams%GaussPriors%std(n))
        BaseParams%PMin = pmin
        BaseParams%PMax = pmax
        BaseParams%center = center
        BaseParams%varying = .false.
        BaseParams%varying(params_used) = .true.
        BaseParams%GaussPriors%mean = pmean
        BaseParams%GaussPriors%std = pstd
        BaseParams%include_fixed_parameter_priors = incl_fixed /= 0
        allocate(BaseParams%LinearCombinations(nlin))
        do k = 1, nlin
            allocate(BaseParams%LinearCombinations(k)%Combination(n))
            read(u_in, *) BaseParams%LinearCombinations(k)%Combination
            read(u_in, *) BaseParams%LinearCombinations(k)%mean, BaseParams%LinearCombinations(k)%std
        end do
        close(u_in)
        Calc%test_likelihood = .true.
        Calc%Temperature = temperature
        allocate(Calc%test_cov_matrix(n_used, n_used))
        Calc%test_cov_matrix = cov       ! TestLikelihoodFunction inverts it (calclike.f90:187-195)
        Pt%P = 0
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
    case ('blocks')
        Feedback = 0
        call BIni%Open(trim(cfg), bad, .false.)
        if (bad) stop 'cannot open blocks config'
        num_params = BIni%Read_Int('num_params')
        num_theory_params = BIni%Read_Int('num_theory_params')
        index_data = num_theory_params + 1
        index_semislow = BIni%Read_Int('index_semislow', -1)
        allocate(ivec(num_params))
        read(BIni%Read_String('varying'), *) ivec
        allocate(BaseParams%varying(num_params))
        BaseParams%varying = ivec /= 0
        num_params_used = count(BaseParams%varying)
        allocate(params_used(num_params_used))
        j = 0
        do i = 1, num_params
            if (BaseParams%varying(i)) then
                j = j + 1
                params_used(j) = i
            end if
        end do
        n = BIni%Read_Int('num_likes')
        DataLikelihoods%first_fast_param = 0
        do i = 1, n
            allocate(TDataLikelihood :: BLike)
            deallocate(ivec)
            allocate(ivec(3))
            read(BIni%Read_String(numcat('like', i)), *) ivec
            BLike%new_param_block_start = ivec(1)
            BLike%new_params = ivec(2)
            BLike%speed = ivec(3)
            call DataLikelihoods%Add(BLike)         ! already in speed order (AddNuisanceParameters sorts)
            if (DataLikelihoods%first_fast_param == 0 .and. BLike%speed >= 0 .and. BLike%new_params > 0) &
                DataLikelihoods%first_fast_param = BLike%new_param_block_start   ! GeneralTypes.f90:650-651
        end do
        call BaseParams%SetFastSlowParams(BIni, BIni%Read_Logical('use_fast_slow', .true.))
        write(u_out, '(*(I6))') size(BaseParams%param_blocks), BaseParams%num_slow, BaseParams%num_fast, &
            BaseParams%num_semi_slow, BaseParams%num_semi_fast
        do i = 1, size(BaseParams%param_blocks)
            write(u_out, '(*(I6))') size(BaseParams%param_blocks(i)%P), BaseParams%param_blocks(i)%P
        end do
    end select
    close(u_out)

contains

    function target(Q) result(L)
        real(mcp), intent(in) :: Q(:)
        real(mcp) :: L
        Pt%P(1:num_params) = Q(1:num_params)
        L = Calc%GetLogLike(Pt)                 ! calclike.f90:136-151
    end function target

end program rng_harness
