"""Weight conversion + golden-model parity against Hugging Face (CPU, fp32).

The reference checked conversions by running the converted model next to the
HF/Meta model (``verify_correctness.py``, ``tests/test_llama_weights.py``).
Here tiny random-init HF Llama / Falcon models (transformers is installed;
no downloads) are converted with ``weights2megatron``, loaded into this
framework at several TP x PP layouts (via ``tools/checkpoint_util.py``) and
their logits compared to HF's; ``megatron2hf`` must round-trip exactly.
"""
import os
import subprocess
import sys

import pytest
import torch

from dist_utils import run_dist, init_framework

transformers = pytest.importorskip("transformers")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "weights2megatron"))


def test_qkv_helpers_roundtrip():
    from epfl_megatron_amd.convert.qkv import pack_qkv, permute_qkv, unpack_qkv
    nq, nkv, hd, h = 8, 2, 16, 128
    wq, wk, wv = torch.randn(nq * hd, h), torch.randn(nkv * hd, h), torch.randn(nkv * hd, h)
    qkv = pack_qkv(wq, wk, wv, nq, nkv)
    assert qkv.shape == ((nq + 2 * nkv) * hd, h)
    # group g = [q_{4g..4g+3}, k_g, v_g]
    torch.testing.assert_close(qkv[4 * hd:5 * hd], wk[:hd])
    for a, b in zip(unpack_qkv(qkv, nq, nkv, hd), (wq, wk, wv)):
        torch.testing.assert_close(a, b)
    p = permute_qkv(qkv, nq * hd, nq, nkv)
    torch.testing.assert_close(permute_qkv(p, nq * hd, nq, nkv, revert=True), qkv)
    # v rows untouched, q rows interleaved: new row 1 = old row hd/2
    torch.testing.assert_close(p[5 * hd:6 * hd], qkv[5 * hd:6 * hd])
    torch.testing.assert_close(p[1], qkv[hd // 2])


def _tiny_llama(path, nkv=2):
    cfg = transformers.LlamaConfig(vocab_size=96, hidden_size=64, intermediate_size=160,
                                   num_attention_heads=4, num_key_value_heads=nkv,
                                   num_hidden_layers=4, max_position_embeddings=64,
                                   rms_norm_eps=1e-5, tie_word_embeddings=False)
    torch.manual_seed(0)
    model = transformers.LlamaForCausalLM(cfg).float().eval()
    with torch.no_grad():
        for p in model.parameters():  # non-trivial norms
            if p.dim() == 1:
                p.add_(0.1 * torch.randn_like(p))
    model.save_pretrained(path, safe_serialization=True)
    return model


def _tiny_falcon(path, new_arch):
    kw = dict(vocab_size=96, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
              parallel_attn=True, bias=False, alibi=False, max_position_embeddings=64)
    if new_arch:
        kw.update(new_decoder_architecture=True, num_kv_heads=2)
    else:
        kw.update(new_decoder_architecture=False, multi_query=True)
    cfg = transformers.FalconConfig(**kw)
    torch.manual_seed(1)
    model = transformers.FalconForCausalLM(cfg).float().eval()
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() == 1:
                p.add_(0.1 * torch.randn_like(p))
    model.save_pretrained(path, safe_serialization=True)
    return model


def _hf_logits(model, tokens):
    with torch.no_grad():
        return model(tokens).logits.float()


def _mega_logits(rank, world, argv, tokens):
    import finetune
    init_framework(argv, finetune.extra_args)
    import torch.distributed as dist
    from epfl_megatron_amd import get_args
    from epfl_megatron_amd.checkpointing import load_checkpoint
    from epfl_megatron_amd.models import ModelType
    from epfl_megatron_amd.parallel import state
    from epfl_megatron_amd.parallel.pipeline import p2p
    from epfl_megatron_amd.training import get_model
    from epfl_megatron_amd.utils.misc import unwrap_model
    args = get_args()
    model = get_model(finetune.model_provider, ModelType.encoder_or_decoder, wrap_with_ddp=False)
    load_checkpoint(model, None, None)
    m = unwrap_model(model)[0].eval()
    b, s = tokens.shape
    with torch.no_grad():
        if not state.is_pipeline_first_stage():
            x = p2p.recv_forward((s, b, args.hidden_size), dtype_=torch.float32)
            m.set_input_tensor(x)
        out = m(tokens, None, None)
        if not state.is_pipeline_last_stage():
            p2p.send_forward(out, (s, b, args.hidden_size), dtype_=torch.float32)
            return None
    tp = state.get_tensor_model_parallel_world_size()
    if tp > 1:
        parts = [torch.empty_like(out) for _ in range(tp)]
        dist.all_gather(parts, out.contiguous(), group=state.get_tensor_model_parallel_group())
        out = torch.cat(parts, dim=-1)
    return out.float()


def _argv_llama(ckpt, tp=1, pp=1, nkv=2):
    return ["--num_layers", "4", "--hidden_size", "64", "--num_attention_heads", "4",
            "--num_attention_heads_kv", str(nkv), "--ffn_hidden_size", "160",
            "--seq_length", "16", "--max_position_embeddings", "64",
            "--position_embedding_type", "rotary", "--use_rms_norm", "--glu_activation",
            "swiglu", "--no_tie_embed_logits", "--layernorm_epsilon", "1e-5",
            "--hidden_dropout", "0.0", "--attention_dropout", "0.0",
            "--no_bias_gelu_fusion", "--no_bias_dropout_fusion",
            "--make_vocab_size_divisible_by", "1", "--synthetic_vocab_size", "96",
            "--model_name", "llama2", "--micro_batch_size", "2", "--global_batch_size", "2",
            "--load", ckpt, "--finetune", "--no_load_optim", "--no_load_rng",
            "--tensor_model_parallel_size", str(tp), "--pipeline_model_parallel_size",
            str(pp), "--use_cpu_initialization", "--train_iters", "1", "--lr", "1e-4"]


def _argv_falcon(ckpt, new_arch, tp=1):
    nkv = 2 if new_arch else 1
    a = ["--num_layers", "2", "--hidden_size", "64", "--num_attention_heads", "4",
         "--num_attention_heads_kv", str(nkv), "--seq_length", "16",
         "--max_position_embeddings", "64", "--position_embedding_type", "rotary",
         "--parallel_attn", "--layernorm_epsilon", "1e-5",
         "--hidden_dropout", "0.0", "--attention_dropout", "0.0",
         "--make_vocab_size_divisible_by", "1", "--synthetic_vocab_size", "96",
         "--model_name", "falcon", "--micro_batch_size", "2", "--global_batch_size", "2",
         "--load", ckpt, "--finetune", "--no_load_optim", "--no_load_rng",
         "--tensor_model_parallel_size", str(tp), "--use_cpu_initialization",
         "--train_iters", "1", "--lr", "1e-4"]
    if new_arch:
        a.append("--parallel_layernorm")
    return a


def _reshard(src, dst, tp, pp, model_type="llama2"):
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "checkpoint_util.py"),
                           "--model_type", model_type, "--load_dir", src, "--save_dir", dst,
                           "--target_tensor_parallel_size", str(tp),
                           "--target_pipeline_parallel_size", str(pp)],
                          stdout=subprocess.DEVNULL)


@pytest.fixture(scope="module")
def llama_ckpt(tmp_path_factory):
    d = tmp_path_factory.mktemp("llama")
    hf = _tiny_llama(str(d / "hf"))
    import weights2megatron as w2m
    w2m.main("llama2", 7, str(d / "mega"), str(d / "hf"))
    tokens = torch.randint(0, 96, (2, 16), generator=torch.Generator().manual_seed(3))
    return d, hf, tokens


def test_llama_hf_logit_parity(llama_ckpt):
    d, hf, tokens = llama_ckpt
    want = _hf_logits(hf, tokens)
    got = [r for r in run_dist(_mega_logits, 1, _argv_llama(str(d / "mega")), tokens)
           if r is not None][0]
    assert got.shape == (2, 16, 96)
    torch.testing.assert_close(got, want, atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("tp,pp", [(2, 1), (1, 2), (2, 2)])
def test_llama_resharded_parity(llama_ckpt, tp, pp):
    d, hf, tokens = llama_ckpt
    dst = str(d / f"mega_tp{tp}_pp{pp}")
    _reshard(str(d / "mega"), dst, tp, pp)
    assert sorted(os.listdir(os.path.join(dst, "release"))) == sorted(
        (f"mp_rank_{r:02d}" if pp == 1 else f"mp_rank_{r:02d}_{p:03d}")
        for r in range(tp) for p in range(pp))
    res = run_dist(_mega_logits, tp * pp, _argv_llama(dst, tp, pp), tokens)
    got = [r for r in res if r is not None][0]
    torch.testing.assert_close(got, _hf_logits(hf, tokens), atol=2e-4, rtol=1e-4)


def test_llama_reshard_roundtrip_exact(llama_ckpt):
    from epfl_megatron_amd.convert.megatron_ckpt import load_full
    d, _, _ = llama_ckpt
    _reshard(str(d / "mega"), str(d / "rt_a"), 2, 2)
    _reshard(str(d / "rt_a"), str(d / "rt_b"), 1, 1)
    _, a, _ = load_full(str(d / "mega"))
    _, b, _ = load_full(str(d / "rt_b"))
    for sect in ("embedding", "transformer"):
        assert a[sect].keys() == b[sect].keys()
        for k in a[sect]:
            assert torch.equal(a[sect][k], b[sect][k]), k
    assert torch.equal(a["lm_head"], b["lm_head"])


def test_megatron2hf_roundtrip(llama_ckpt, tmp_path):
    d, hf, tokens = llama_ckpt
    import megatron2hf
    _reshard(str(d / "mega"), str(d / "m2h_src"), 2, 1)  # sharded input is accepted
    megatron2hf.main(["--input_dir", str(d / "m2h_src"), "--output_dir", str(tmp_path / "out"),
                      "--model", "llama2", "--no_tokenizer"])
    back = transformers.LlamaForCausalLM.from_pretrained(str(tmp_path / "out")).float().eval()
    ref = hf.state_dict()
    for k, v in back.state_dict().items():
        assert torch.equal(v, ref[k]), k
    torch.testing.assert_close(_hf_logits(back, tokens), _hf_logits(hf, tokens))


@pytest.mark.parametrize("new_arch", [False, True])
def test_falcon_hf_logit_parity(tmp_path, new_arch):
    hf = _tiny_falcon(str(tmp_path / "hf"), new_arch)
    import weights2megatron as w2m
    w2m.main("falcon", 7, str(tmp_path / "mega"), str(tmp_path / "hf"))
    tokens = torch.randint(0, 96, (2, 16), generator=torch.Generator().manual_seed(4))
    want = _hf_logits(hf, tokens)
    got = run_dist(_mega_logits, 1, _argv_falcon(str(tmp_path / "mega"), new_arch), tokens)[0]
    torch.testing.assert_close(got, want, atol=2e-4, rtol=1e-4)
    if new_arch:  # TP=2 splits the 2 KV groups
        _reshard(str(tmp_path / "mega"), str(tmp_path / "tp2"), 2, 1, "falcon")
        res = run_dist(_mega_logits, 2, _argv_falcon(str(tmp_path / "tp2"), new_arch, 2), tokens)
        torch.testing.assert_close(res[0], want, atol=2e-4, rtol=1e-4)
    import megatron2hf
    megatron2hf.main(["--input_dir", str(tmp_path / "mega"), "--output_dir",
                      str(tmp_path / "back"), "--model", "falcon", "--no_tokenizer"])
    back = transformers.FalconForCausalLM.from_pretrained(str(tmp_path / "back")).float().eval()
    torch.testing.assert_close(_hf_logits(back, tokens), want)


def _verify(rank, world, ckpt, hfdir):
    import verify_correctness as vc
    from dist_utils import init_framework
    argv = ["--model_name", "llama2", "--load", ckpt, "--huggingface_cache", hfdir,
            "--huggingface_device", "cpu", "--synthetic_data", "--tokenizer_type",
            "NullTokenizer", "--synthetic_vocab_size", "96", "--make_vocab_size_divisible_by",
            "1", "--seq_length", "16", "--use_cpu_initialization", "--global_batch_size", "1",
            "--no_bias_gelu_fusion", "--no_bias_dropout_fusion", "--hidden_dropout", "0.0",
            "--attention_dropout", "0.0", "--eval_iters", "0"]
    from epfl_megatron_amd.initialize import initialize_megatron
    initialize_megatron(vc.extra_extra_args, vc.defaults_for(ckpt),
                        args_list=["--distributed_backend", "gloo", "--num_workers", "0"] + argv)
    return vc.main(iters=2)


def test_verify_correctness_cli(llama_ckpt):
    d, _, _ = llama_ckpt
    res = run_dist(_verify, 1, str(d / "mega"), str(d / "hf"))[0]
    assert len(res) == 2
    for max_err, loss_err in res:
        assert max_err < 1e-3 and loss_err < 1e-4


def _hf_to_meta_layout(w, n_heads):
    """HF rotate-half rows -> Meta interleaved rows (inverse of HF's own permute)."""
    hd = w.shape[0] // n_heads
    return w.view(n_heads, 2, hd // 2, w.shape[1]).transpose(1, 2).reshape(w.shape)


def test_convert_llama2hf_from_meta_shards(llama_ckpt, tmp_path):
    """Tiny HF model -> genuine 2-way Meta shards -> convert_llama2hf -> same HF weights."""
    import json
    import convert_llama2hf
    from epfl_megatron_amd.convert.llama import META_SHARD_DIM, hf_to_meta
    d, hf, tokens = llama_ckpt
    meta = hf_to_meta(hf.state_dict())
    for k in list(meta):
        if k.endswith("attention.wq.weight"):
            meta[k] = _hf_to_meta_layout(meta[k], 4)
        elif k.endswith("attention.wk.weight"):
            meta[k] = _hf_to_meta_layout(meta[k], 2)
    src = tmp_path / "meta" / "7B"
    src.mkdir(parents=True)
    for r in range(2):
        shard = {}
        for k, v in meta.items():
            dim = META_SHARD_DIM[k.split(".")[-2]]
            shard[k] = v.clone() if dim is None else torch.chunk(v, 2, dim=dim)[r].clone()
        torch.save(shard, src / f"consolidated.{r:02d}.pth")
    (src / "params.json").write_text(json.dumps({"dim": 64, "n_layers": 4, "n_heads": 4,
                                                 "n_kv_heads": 2, "norm_eps": 1e-5,
                                                 "vocab_size": 96}))
    out = tmp_path / "hf_out"
    convert_llama2hf.main(["--input_dir", str(tmp_path / "meta"), "--model_size", "7B",
                           "--output_dir", str(out)])
    back = transformers.LlamaForCausalLM.from_pretrained(str(out)).float().eval()
    ref = hf.state_dict()
    for k, v in back.state_dict().items():
        assert torch.equal(v, ref[k]), k
    torch.testing.assert_close(_hf_logits(back, tokens), _hf_logits(hf, tokens))
