"""GLUE (MNLI / QQP) classification finetuning (reference ``tasks/glue/finetune.py``)."""
from epfl_megatron_amd import get_args, get_tokenizer, print_rank_0
from epfl_megatron_amd.models import Classification, ModelType

from ..eval_utils import accuracy_func_provider
from ..finetune_utils import finetune
from .data import MNLIDataset, QQPDataset

_TASKS = {"MNLI": (3, MNLIDataset), "QQP": (2, QQPDataset)}


def name_from_datapath(task, datapath):
    """``.../MNLI/dev_matched.tsv`` -> ``dev-matched`` (reference naming; note
    ``str.strip('.tsv')`` strips characters, not a suffix)."""
    return datapath.split(task)[-1].strip(".tsv").strip("/").replace("_", "-")


def glue_classification(task):
    num_classes, Dataset = _TASKS[task]

    def train_valid_datasets_provider():
        args, tok = get_args(), get_tokenizer()
        return (Dataset("training", args.train_data, tok, args.seq_length),
                Dataset("validation", args.valid_data, tok, args.seq_length))

    def model_provider(pre_process=True, post_process=True):
        print_rank_0(f"building classification model for {task} ...")
        return Classification(num_classes=num_classes, num_tokentypes=2,
                              pre_process=pre_process, post_process=post_process,
                              model_type=ModelType.encoder_or_decoder)

    def metrics_func_provider():
        def single(datapath):
            args = get_args()
            return Dataset(name_from_datapath(task, datapath), [datapath], get_tokenizer(),
                           args.seq_length)
        return accuracy_func_provider(single)

    return finetune(train_valid_datasets_provider, model_provider, ModelType.encoder_or_decoder,
                    end_of_epoch_callback_provider=metrics_func_provider)


def main():
    task = get_args().task
    if task not in _TASKS:
        raise NotImplementedError(f"GLUE task {task} is not implemented.")
    return glue_classification(task)
