"""Number-of-microbatches calculators (reference ``megatron/microbatches.py``).

``num_microbatches = global_batch / (micro_batch * data_parallel)``, optionally
with a linear global-batch ramp-up driven by the number of consumed samples.
"""


class MicroBatchCalculator:
    def __init__(self, micro_batch_size, data_parallel_size):
        self.micro_batch_size = micro_batch_size
        self.data_parallel_size = data_parallel_size
        self.micro_batch_times_data_parallel_size = micro_batch_size * data_parallel_size
        self.num_micro_batches = None
        self.current_global_batch_size = None

    def get(self):
        return self.num_micro_batches

    def get_current_global_batch_size(self):
        return self.current_global_batch_size

    def update(self, consumed_samples, consistency_check):
        raise NotImplementedError


class ConstantNumMicroBatches(MicroBatchCalculator):
    def __init__(self, global_batch_size, micro_batch_size, data_parallel_size):
        super().__init__(micro_batch_size, data_parallel_size)
        per_step = self.micro_batch_times_data_parallel_size
        if global_batch_size % per_step != 0:
            raise AssertionError(
                f"global batch size ({global_batch_size}) is not divisible by micro batch size "
                f"({micro_batch_size}) times data parallel size ({data_parallel_size})")
        self.num_micro_batches = global_batch_size // per_step
        if self.num_micro_batches < 1:
            raise AssertionError("number of micro-batches should be at least 1")
        self.current_global_batch_size = global_batch_size

    def update(self, consumed_samples, consistency_check):
        return None


class RampupBatchsizeNumMicroBatches(MicroBatchCalculator):
    """Linearly grow the global batch from ``start`` by ``increment`` over
    ``ramup_samples`` consumed samples, then hold ``global_batch_size``."""

    def __init__(self, start_batch_size, batch_size_increment, ramup_samples,
                 global_batch_size, micro_batch_size, data_parallel_size):
        super().__init__(micro_batch_size, data_parallel_size)
        self.start_batch_size = start_batch_size
        self.global_batch_size = global_batch_size
        self.batch_size_increment = batch_size_increment
        self.ramup_samples = ramup_samples
        if start_batch_size <= 0 or batch_size_increment <= 0 or ramup_samples < 0:
            raise AssertionError("invalid ramp-up parameters")
        diff = global_batch_size - start_batch_size
        if diff < 0 or diff % batch_size_increment != 0:
            raise AssertionError("expected global batch size interval to be divisible by the "
                                 "batch size increment")
        steps = diff // batch_size_increment
        self.rampup_samples_per_increment = self.ramup_samples / max(steps, 1)
        self.update(0, False)

    def update(self, consumed_samples, consistency_check):
        if consumed_samples > self.ramup_samples:
            gbs = self.global_batch_size
        else:
            steps = int(consumed_samples / self.rampup_samples_per_increment)
            gbs = self.start_batch_size + steps * self.batch_size_increment
            gbs = min(gbs, self.global_batch_size)
        self.current_global_batch_size = gbs
        if consistency_check and gbs % self.micro_batch_times_data_parallel_size != 0:
            raise AssertionError(f"current global batch size ({gbs}) is not divisible by "
                                 f"micro-batch-size times data parallel size")
        self.num_micro_batches = gbs // self.micro_batch_times_data_parallel_size


def build_num_microbatches_calculator(args):
    if args.rampup_batch_size is None:
        calc = ConstantNumMicroBatches(args.global_batch_size, args.micro_batch_size,
                                       args.data_parallel_size)
        if args.rank == 0:
            print(f"setting number of micro-batches to constant {calc.get()}", flush=True)
        return calc
    if len(args.rampup_batch_size) != 3:
        raise AssertionError("expected --rampup_batch_size <start> <increment> <samples>")
    start, incr, samples = (int(v) for v in args.rampup_batch_size)
    if args.rank == 0:
        print(f"will use batch size rampup starting from global batch size {start} to "
              f"global batch size {args.global_batch_size} with batch size increments "
              f"{incr} over {samples} samples.", flush=True)
    return RampupBatchsizeNumMicroBatches(start, incr, samples, args.global_batch_size,
                                          args.micro_batch_size, args.data_parallel_size)
