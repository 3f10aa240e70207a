"""Tokenizers (reference ``megatron/tokenizer/tokenizer.py``).

Same ``--tokenizer_type`` names and — important for checkpoint/data
compatibility — the same special-token id assignment order for
SentencePiece (``<CLS> <SEP> <EOD> <MASK>`` pad bos eos extra-ids extra-list,
appended after the base vocab unless ``--no_new_tokens``).  GPT-2 BPE, BERT
WordPiece and Falcon use the HuggingFace ``transformers`` implementations
from local vocab files (no network).  ``NullTokenizer`` serves synthetic data.
"""
from abc import ABC, abstractmethod


def build_tokenizer(args):
    if args.rank == 0:
        print(f"> building {args.tokenizer_type} tokenizer ...", flush=True)
    t = args.tokenizer_type
    if t not in ("FalconTokenizer", "NullTokenizer") and args.vocab_file is None:
        raise AssertionError("--vocab_file is required for this tokenizer type")
    if t == "BertWordPieceLowerCase":
        tok = BertWordPieceTokenizer(args.vocab_file, lower_case=True,
                                     vocab_extra_ids=args.vocab_extra_ids)
    elif t == "BertWordPieceCase":
        tok = BertWordPieceTokenizer(args.vocab_file, lower_case=False,
                                     vocab_extra_ids=args.vocab_extra_ids)
    elif t == "GPT2BPETokenizer":
        if args.merge_file is None:
            raise AssertionError("--merge_file is required for GPT2BPETokenizer")
        tok = GPT2BPETokenizer(args.vocab_file, args.merge_file)
    elif t == "SentencePieceTokenizer":
        tok = SentencePieceTokenizer(args.vocab_file, vocab_extra_ids=args.vocab_extra_ids,
                                     vocab_extra_ids_list=args.vocab_extra_ids_list,
                                     new_tokens=args.new_tokens)
    elif t == "FalconTokenizer":
        tok = FalconTokenizer(args.tokenizer_model or args.vocab_file or "tiiuae/falcon-40b",
                              vocab_extra_ids_list=args.vocab_extra_ids_list,
                              new_tokens=args.new_tokens)
    elif t == "NullTokenizer":
        tok = NullTokenizer(args.synthetic_vocab_size)
    else:
        raise NotImplementedError(f"{t} tokenizer is not implemented.")
    args.padded_vocab_size = vocab_size_with_padding(tok.vocab_size, args)
    return tok


def vocab_size_with_padding(orig_vocab_size, args):
    """Round up to a multiple of make_vocab_size_divisible_by * TP."""
    tp = getattr(args, "simulated_tensor_parallel_size", None) or args.tensor_model_parallel_size
    multiple = args.make_vocab_size_divisible_by * tp
    after = ((orig_vocab_size + multiple - 1) // multiple) * multiple
    if args.rank == 0:
        print(f" > padded vocab (size: {orig_vocab_size}) with {after - orig_vocab_size} dummy "
              f"tokens (new size: {after})", flush=True)
    return after


_vocab_size_with_padding = vocab_size_with_padding


class AbstractTokenizer(ABC):
    def __init__(self, name):
        self.name = name

    @property
    @abstractmethod
    def vocab_size(self):
        ...

    @property
    @abstractmethod
    def vocab(self):
        ...

    @property
    @abstractmethod
    def inv_vocab(self):
        ...

    @abstractmethod
    def tokenize(self, text):
        ...

    def detokenize(self, token_ids):
        raise NotImplementedError(f"detokenizer is not implemented for {self.name} tokenizer")

    @property
    def cls(self):
        raise NotImplementedError(f"CLS is not provided for {self.name} tokenizer")

    @property
    def sep(self):
        raise NotImplementedError(f"SEP is not provided for {self.name} tokenizer")

    @property
    def pad(self):
        raise NotImplementedError(f"PAD is not provided for {self.name} tokenizer")

    @property
    def eod(self):
        raise NotImplementedError(f"EOD is not provided for {self.name} tokenizer")

    @property
    def mask(self):
        raise NotImplementedError(f"MASK is not provided for {self.name} tokenizer")


class NullTokenizer(AbstractTokenizer):
    """Integer 'tokens' for synthetic data; the last id is EOD."""

    def __init__(self, vocab_size):
        super().__init__("NullTokenizer")
        self._n = int(vocab_size)

    @property
    def vocab_size(self):
        return self._n

    @property
    def vocab(self):
        return {str(i): i for i in range(self._n)}

    @property
    def inv_vocab(self):
        return {i: str(i) for i in range(self._n)}

    def tokenize(self, text):
        return [int(x) for x in text.split()]

    def detokenize(self, ids):
        return " ".join(str(int(x)) for x in ids)

    @property
    def eod(self):
        return self._n - 1


class GPT2BPETokenizer(AbstractTokenizer):
    def __init__(self, vocab_file, merge_file):
        super().__init__("GPT2 BPE")
        from .gpt2_bpe import GPT2BPE
        self.tokenizer = GPT2BPE(vocab_file, merge_file, errors="replace")
        self.eod_id = self.tokenizer.encoder["<|endoftext|>"]

    @property
    def vocab_size(self):
        return len(self.tokenizer.encoder)

    @property
    def vocab(self):
        return self.tokenizer.encoder

    @property
    def inv_vocab(self):
        return self.tokenizer.decoder

    def tokenize(self, text):
        return self.tokenizer.encode(text)

    def detokenize(self, token_ids):
        return self.tokenizer.decode(token_ids)

    @property
    def eod(self):
        return self.eod_id


class BertWordPieceTokenizer(AbstractTokenizer):
    def __init__(self, vocab_file, lower_case=True, vocab_extra_ids=0):
        super().__init__("BERT Lower Case" if lower_case else "BERT Upper Case")
        from transformers import BertTokenizer
        self.tokenizer = BertTokenizer(vocab_file, do_lower_case=lower_case)
        v = self.tokenizer.vocab
        self.cls_id, self.sep_id = v["[CLS]"], v["[SEP]"]
        self.pad_id, self.mask_id = v["[PAD]"], v["[MASK]"]
        self._additional_special_tokens = []
        extra = {"eos_token": "[EOS]", "bos_token": "[BOS]"}
        self._bos_token, self._eos_token = "[BOS]", "[EOS]"
        self.tokenizer.add_special_tokens(extra)
        extra_ids = [f"<extra_id_{i}>" for i in range(vocab_extra_ids)]
        if extra_ids:
            self.tokenizer.add_special_tokens({"additional_special_tokens": extra_ids})
            self._additional_special_tokens = extra_ids

    @property
    def vocab_size(self):
        return len(self.tokenizer)

    @property
    def vocab(self):
        return self.tokenizer.get_vocab()

    @property
    def inv_vocab(self):
        # id order (HF's get_vocab() orders added tokens nondeterministically
        # across processes; BERT/T5 masking draws random ids from this list)
        return {i: t for t, i in sorted(self.tokenizer.get_vocab().items(), key=lambda kv: kv[1])}

    def tokenize(self, text):
        return self.tokenizer.convert_tokens_to_ids(self.tokenizer.tokenize(text))

    def decode(self, ids):
        return self.tokenizer.decode(ids)

    def detokenize(self, ids):
        return self.tokenizer.decode(ids)

    def decode_token_ids(self, token_ids):
        toks = self.tokenizer.convert_ids_to_tokens(token_ids)
        out = " ".join(t for t in toks if t not in ("[PAD]", "[CLS]"))
        return out.replace(" ##", "").replace("##", "")

    @property
    def cls(self):
        return self.cls_id

    @property
    def sep(self):
        return self.sep_id

    @property
    def pad(self):
        return self.pad_id

    @property
    def mask(self):
        return self.mask_id

    @property
    def bos_token_id(self):
        return self.tokenizer.convert_tokens_to_ids(self._bos_token)

    @property
    def eos_token_id(self):
        return self.tokenizer.convert_tokens_to_ids(self._eos_token)

    @property
    def eod(self):
        return self.eos_token_id

    @property
    def additional_special_tokens_ids(self):
        return [self.tokenizer.convert_tokens_to_ids(t) for t in self._additional_special_tokens]


class FalconTokenizer(AbstractTokenizer):
    def __init__(self, path, vocab_extra_ids_list=None, new_tokens=True):
        super().__init__("FalconTokenizer")
        from transformers import AutoTokenizer
        self.tokenizer = AutoTokenizer.from_pretrained(path)
        self._eod = self.tokenizer.vocab["<|endoftext|>"]
        if vocab_extra_ids_list and new_tokens:
            self.tokenizer.add_special_tokens({"additional_special_tokens":
                                               self.tokenizer.additional_special_tokens
                                               + vocab_extra_ids_list.split(",")})
        self._inv_vocab = {i: t for t, i in self.tokenizer.vocab.items()}

    @property
    def vocab_size(self):
        return len(self.tokenizer.vocab)

    @property
    def vocab(self):
        return self.tokenizer.vocab

    @property
    def inv_vocab(self):
        return self._inv_vocab

    def tokenize(self, text):
        return self.tokenizer.encode(text)

    def detokenize(self, token_ids):
        return self.tokenizer.decode(token_ids)

    @property
    def eod(self):
        return self._eod


class SentencePieceTokenizer(AbstractTokenizer):
    """SentencePiece + Megatron special tokens (ids appended after the base vocab)."""

    def __init__(self, model_file, vocab_extra_ids=0, vocab_extra_ids_list=None, new_tokens=True):
        super().__init__("SentencePieceTokenizer")
        import sentencepiece
        self._tokenizer = sentencepiece.SentencePieceProcessor(model_file=model_file)
        self._vocab, self._inv_vocab = {}, {}
        self._special_tokens, self._inv_special_tokens = {}, {}
        self._t5_tokens = []
        for i in range(len(self._tokenizer)):
            piece = self._tokenizer.id_to_piece(i)
            self._inv_vocab[i] = piece
            self._vocab[piece] = i
        self._new_tokens = new_tokens

        def piece_or(fn, fallback):
            try:
                return self._tokenizer.id_to_piece(fn())
            except IndexError:
                return fallback

        names = ["<CLS>", "<SEP>", "<EOD>", "<MASK>",
                 piece_or(self._tokenizer.pad_id, "<PAD>"),
                 piece_or(self._tokenizer.bos_id, "<BOS>"),
                 piece_or(self._tokenizer.eos_id, "<EOS>")]
        ids = [self._add_special(n) for n in names]
        (self._cls_id, self._sep_id, self._eod_id, self._mask_id, self._pad_id, self._bos_id,
         self._eos_id) = ids
        for i in range(vocab_extra_ids):
            t = f"<extra_id_{i}>"
            self._add_special(t)
            self._t5_tokens.append(t)
        if vocab_extra_ids_list:
            for t in vocab_extra_ids_list.split(","):
                self._add_special(t)
        print(f"Special tokens: {self._special_tokens}")

    def _add_special(self, t):
        if t not in self._vocab and not self._new_tokens:
            return self._vocab.get(t)
        if t not in self._vocab:
            nid = len(self._vocab)
            self._vocab[t] = nid
            self._inv_vocab[nid] = t
        self._special_tokens[t] = self._vocab[t]
        self._inv_special_tokens[self._vocab[t]] = t
        return self._vocab[t]

    @property
    def vocab_size(self):
        return len(self._vocab)

    @property
    def vocab(self):
        return self._vocab

    @property
    def inv_vocab(self):
        return self._inv_vocab

    def tokenize(self, text):
        """Split on special tokens (earliest match first), SentencePiece in between."""
        ids, pos = [], 0
        while True:
            best, best_at = None, None
            for tok in self._special_tokens:
                at = text.find(tok, pos)
                if at >= 0 and (best_at is None or at < best_at):
                    best, best_at = tok, at
            if best is None:
                break
            ids.extend(self._tokenizer.encode_as_ids(text[pos:best_at]))
            ids.append(self._special_tokens[best])
            pos = best_at + len(best)
        ids.extend(self._tokenizer.encode_as_ids(text[pos:]))
        return ids

    def detokenize(self, ids):
        out, last = "", 0
        for i, tid in enumerate(ids):
            if tid in self._inv_special_tokens:
                out += self._tokenizer.decode_ids(ids[last:i]) + " "
                out += self._inv_special_tokens[tid] + " "
                last = i + 1
        out += self._tokenizer.decode_ids(ids[last:])
        return out.strip()

    @property
    def cls(self):
        return self._cls_id

    @property
    def sep(self):
        return self._sep_id

    @property
    def pad(self):
        return self._pad_id

    @property
    def bos_token_id(self):
        return self._bos_id

    @property
    def bos(self):
        return self._bos_id

    @property
    def eod(self):
        return self._eod_id if self._eod_id is not None else self._eos_id

    @property
    def eos_token_id(self):
        return self.eod

    @property
    def eos(self):
        return self._eos_id

    @property
    def mask(self):
        return self._mask_id

    @property
    def additional_special_tokens_ids(self):
        return [self.vocab[k] for k in self._t5_tokens]
