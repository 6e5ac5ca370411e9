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
!   mode "chain"  : the reference's own sampler loop (module MonteCarlo,
!                   MCMC.f90) on the test_likelihood Gaussian:
!                   TMetropolisSampler_GetNewSample (:269-307), FastParameterSample
!                   (:309-335) or TFastDraggingSampler_GetNewSample (:338-452)
!                   with its MetropolisAccept (:119-131) and MoveDone (:166-190),
!                   the reference's BlockedProposer, and every -lnL from the
!                   reference's TLikeCalculator%GetLogLike (calclike.f90:136-151:
!                   hard bounds :97-109, TestLikelihoodFunction :180-199, Gaussian
!                   and linear-combination priors with the
!                   include_fixed_parameter_priors gate :111-134, temperature
!                   :82-94); num_params may exceed num_params_used (fixed
!                   parameters).  MoveDone's AddNewWeightedPoint goes to the
!                   reference's TMpiChainCollector (SampleCollector.f90:82-112),
!                   which writes the chain file rows.  Two recorders (module
!                   harness_recorders below) only observe: the MetropolisAccept
!                   override logs the last decision and its -lnL argument, the
!                   collector override logs each AddNewWeightedPoint call.
!   mode "blocks" : TBaseParameters_SetFastSlowParams (BaseParameters.f90:302-433)
!                   on BaseParams%varying and a DataLikelihoods list of plain
!                   TDataLikelihood items carrying new_param_block_start /
!                   new_params / speed, the blocking keys read from the config
!                   itself (an ini file); writes every param_blocks entry
!
! usage: rng_harness kat|stream|chain|gr|confid|blocks <config> <out.txt>
module harness_recorders
    ! Observers over the reference's own types: each override records its
    ! arguments/result and defers to the reference procedure unchanged.
    use settings
    use GeneralTypes
    use CalcLike
    use MonteCarlo
    use SampleCollector
    implicit none

    ! TFastDraggingSampler_GetNewSample calls this%TMetropolisSampler%FastParameterSample
    ! (MCMC.f90:359), a non-polymorphic parent call, so the MetropolisAccept override
    ! is not reached from the fast sub-steps of dragging: the harness takes a step's
    ! accept from the point moving, its trial -lnL from the override when it fired
    ! (the drag's DragLike, :438) and otherwise from the calculator's last value.
    Type, extends(TFastDraggingSampler) :: TRecSampler
        logical :: fired = .false.
        real(mcp) :: last_like = LogZero
    contains
    procedure :: MetropolisAccept => Rec_MetropolisAccept
    end Type

    Type, extends(TGenericLikeCalculator) :: TRecCalc
        real(mcp) :: last_like = LogZero
    contains
    procedure :: GetLogLike => Rec_GetLogLike
    end Type

    Type, extends(TMpiChainCollector) :: TRecCollector
        integer :: u_points = 0
    contains
    procedure :: AddNewWeightedPoint => Rec_AddNewWeightedPoint
    end Type

contains

    function Rec_MetropolisAccept(this, Like, CurLike) result(MetropolisAccept)
    class(TRecSampler) :: this
    real(mcp) Like, CurLike
    logical MetropolisAccept

    MetropolisAccept = this%TChainSampler%MetropolisAccept(Like, CurLike)
    this%fired = .true.
    this%last_like = Like

    end function Rec_MetropolisAccept

    function Rec_GetLogLike(this, Params) result(L)
    class(TRecCalc) :: this
    class(TCalculationAtParamPoint) :: Params
    real(mcp) L

    L = this%TGenericLikeCalculator%GetLogLike(Params)
    this%last_like = L

    end function Rec_GetLogLike

    subroutine Rec_AddNewWeightedPoint(this, CurParams, CurLike, mult, thin_fac)
    class(TRecCollector) :: this
    class(TCalculationAtParamPoint), intent(in) :: CurParams
    real(mcp) CurLike
    real(mcp), intent(in):: mult
    integer, intent(in), optional :: thin_fac
    integer thin

    thin = 1
    if (present(thin_fac)) thin = thin_fac
    write(this%u_points, '(2I6,*(ES25.17))') nint(mult), thin, CurLike, CurParams%P(params_used)
    call this%TMpiChainCollector%AddNewWeightedPoint(CurParams, CurLike, mult, thin_fac)

    end subroutine Rec_AddNewWeightedPoint

end module harness_recorders

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
    use ParamPointSet
    use harness_recorders
    implicit none
    character(LEN=1024) :: mode, cfg, outf
    integer :: u_in, u_out, i, j, k, n, nsteps, nblocks, slow_block_max, oversample, ij, kl, nrot
    integer :: fast_only, nidx
    real(mcp) :: scale, like, curlike, temperature
    real(mcp), allocatable :: cov(:,:), covinv(:,:), P(:), trial(:), center(:), pmin(:), pmax(:)
    real(mcp), allocatable :: pmean(:), pstd(:), R(:,:), X(:)
    integer, allocatable :: bsize(:), ind(:)
    type(int_arr), allocatable :: blocks(:)
    logical :: accpt
    real :: e
    real(mcp), allocatable :: mcov(:,:), evals(:)
    real(mcp) :: mult
    integer :: n_used, incl_fixed, nlin, ix1, ix2, burn
    Type(TSampleList) :: SL
    real(mcp) :: limfrac, lower, upper
    Type(TRecCalc), target :: Calc
    Type(TRecSampler) :: Sampler
    Type(TRecCollector), target :: Collector
    Type(TGeneralConfig), target :: GConfig
    Type(GenericParameterization), target :: Gp
    Type(ParamSet) :: CurParams
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
        ! The reference's own sampler loop (module MonteCarlo, MCMC.f90) on the
        ! test_likelihood Gaussian: fast_only 0 -> TMetropolisSampler_GetNewSample
        ! (:269-307), 1 -> FastParameterSample (:309-335), 2 ->
        ! TFastDraggingSampler_GetNewSample (:338-452).  MoveDone (:166-190)
        ! feeds the reference's TMpiChainCollector_AddNewWeightedPoint
        ! (SampleCollector.f90:82-112), which writes the chain file rows through
        ! WriteParams / IO_OutputChainRow into <out>.txt; <out>.points logs each
        ! AddNewWeightedPoint call at full precision, <out>.max the MaxLike.
        open(newunit=u_in, file=trim(cfg), status='old')
        read(u_in, *) ij, kl, n, n_used, nsteps, fast_only, incl_fixed, nlin
        read(u_in, *) nblocks, slow_block_max, oversample, scale, temperature, burn
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
        allocate(cov(n_used,n_used), P(n), center(n), pmin(n), pmax(n), pmean(n), pstd(n))
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
        ! param_blocks as SetFastSlowParams lays them out: entries 1..slow_tp_max (= 2) are the
        ! slow types (empty ones skipped by BlockedProposer%Init, propose.f90:170-180), then fast
        if (slow_block_max > slow_tp_max) stop 'chain: more than slow_tp_max slow blocks'
        allocate(BaseParams%param_blocks(nblocks + slow_tp_max - slow_block_max))
        j = 0
        BaseParams%num_slow = 0
        BaseParams%num_fast = 0
        do i = 1, nblocks
            j = j + 1
            if (i == slow_block_max + 1) then
                do k = slow_block_max + 1, slow_tp_max
                    allocate(BaseParams%param_blocks(j)%P(0))
                    j = j + 1
                end do
            end if
            allocate(BaseParams%param_blocks(j)%P(bsize(i)))
            BaseParams%param_blocks(j)%P = blocks(i)%P
            if (i <= slow_block_max) then
                BaseParams%num_slow = BaseParams%num_slow + bsize(i)
            else
                BaseParams%num_fast = BaseParams%num_fast + bsize(i)
            end if
        end do
        do while (j < size(BaseParams%param_blocks))
            j = j + 1
            allocate(BaseParams%param_blocks(j)%P(0))
        end do
        Calc%test_likelihood = .true.
        Calc%Temperature = temperature
        allocate(Calc%test_cov_matrix(n_used, n_used))
        Calc%test_cov_matrix = cov       ! TestLikelihoodFunction inverts it (calclike.f90:187-195)
        GConfig%Parameterization => Gp
        Collector%Config => GConfig
        open(newunit=Collector%u_points, file=trim(outf)//'.points', status='replace')
        call ChainOutFile%CreateFile(trim(outf)//'.txt')
        call initRandom(ij, kl)
        Sampler%oversample_fast = oversample
        Sampler%burn_in = burn
        call Sampler%InitWithPropose(Calc, Collector, propose_scale=scale)
        call Sampler%SetCovariance(cov)
        CurParams%P = 0
        CurParams%P(1:n) = P
        curlike = Sampler%LogLike(CurParams)
        write(u_out, '(ES25.17)') curlike
        mult = 0                                    ! TChainSampler_SampleFrom (MCMC.f90:141)
        allocate(trial(n))
        do k = 1, nsteps
            Sampler%fired = .false.
            Calc%last_like = LogZero
            trial = CurParams%P(1:n)
            select case (fast_only)
            case (0)
                call Sampler%GetNewMetropolisSample(CurParams, curlike, mult)
            case (1)
                call Sampler%FastParameterSample(CurParams, curlike, mult)
            case default
                call Sampler%GetNewSample(CurParams, curlike, mult)
            end select
            if (.not. Sampler%fired) Sampler%last_like = Calc%last_like
            write(u_out, '(I2,*(ES25.17))') merge(1, 0, any(CurParams%P(1:n) /= trial)), Sampler%last_like, &
                curlike, CurParams%P(1:n)
        end do
        call ChainOutFile%Close()
        close(Collector%u_points)
        open(newunit=u_in, file=trim(outf)//'.max', status='replace')
        write(u_in, '(I8,*(ES25.17))') Sampler%num_accept, Sampler%MaxLike, Sampler%MaxLikeParams(1:n)
        close(u_in)
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

end program rng_harness
