"""RACE multiple-choice finetuning (reference ``tasks/race/finetune.py``)."""
from epfl_megatron_amd import get_args, get_tokenizer, print_rank_0
from epfl_megatron_amd.models import ModelType, MultipleChoice

from ..eval_utils import accuracy_func_provider
from ..finetune_utils import finetune
from .data import RaceDataset


def train_valid_datasets_provider():
    args, tok = get_args(), get_tokenizer()
    return (RaceDataset("training", args.train_data, tok, args.seq_length),
            RaceDataset("validation", args.valid_data, tok, args.seq_length))


def model_provider(pre_process=True, post_process=True):
    print_rank_0("building multichoice model for RACE ...")
    return MultipleChoice(num_tokentypes=2, pre_process=pre_process, post_process=post_process,
                          model_type=ModelType.encoder_or_decoder)


def metrics_func_provider():
    def single(datapath):
        name = datapath.split("RACE")[-1].strip("/").replace("/", "-")
        return RaceDataset(name, [datapath], get_tokenizer(), get_args().seq_length)
    return accuracy_func_provider(single)


def main():
    return finetune(train_valid_datasets_provider, model_provider, ModelType.encoder_or_decoder,
                    end_of_epoch_callback_provider=metrics_func_provider)
