"""MSDP-EVAL-F1 (reference ``tasks/msdp/evaluate.py:11-45``): F1 of a generated
file against a golden file, line by line."""
from epfl_megatron_amd import get_args, print_rank_0

from .metrics import F1Metric

EOD_TEXT = "<|endoftext|>"


def read_guesses(path):
    with open(path) as f:
        return [line.strip().replace(EOD_TEXT, "") for line in f]


def read_answers(path):
    with open(path) as f:
        return ["" if line.strip() == "no_passages_used" else line.strip() for line in f]


def evaluate_f1(guess_file, answer_file):
    guesses, answers = read_guesses(guess_file), read_answers(answer_file)
    assert len(guesses) == len(answers), "lengths of guess and answer are different!"
    p, r, f1 = F1Metric.compute_all_pairs(guesses, answers)
    print_rank_0("Precision: %.4f; recall: %.4f; f1: %.4f" % (p, r, f1))
    return p, r, f1


def main():
    args = get_args()
    return evaluate_f1(args.guess_file, args.answer_file)
