"""Training path on CPU: differentiable forwards match the serving forwards, LoRA starts at
the base model and merges exactly, SFT loss falls, checkpoint/resume is step-exact, and
2-rank data parallelism (gloo, bucketed all-reduce) equals one rank on the whole batch."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from nv_genai_amd.models.config import encoder_config, llama_config


def _llama(seed=0):
    from nv_genai_amd.models.llama import LlamaModel

    cfg = llama_config("llama-tiny", layers=2, max_position=256)
    return LlamaModel(cfg, "cpu", seed=seed)


class CharTok:
    def encode(self, s):
        return [3 + (ord(c) % 200) for c in s]


DATA = [{"input": f"question {i}: what is {i} plus one?", "output": f" {i + 1}"} for i in range(16)]


def test_llama_training_forward_matches_serving():
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.training import functional as Fn

    m = _llama()
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=2, max_batched_tokens=256, max_model_len=256,
                                 kv_cache_blocks=8, use_graphs=False), device="cpu", model=m, model_cfg=m.cfg)
    torch.manual_seed(1)
    ids = torch.randint(0, 30000, (1, 37))
    out = eng.generate([ids[0].tolist()], SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))[0].output_ids
    full = torch.cat([ids, torch.tensor([out[:2]])], 1)
    lg = Fn.llama_hidden(m, full)[0].float() @ m.lm_head.float().t()
    # bf16 near-ties may flip the argmax between the two op sets: the served token must be
    # (near-)top under the training forward
    top = lg[-3:].topk(3, dim=-1).indices.tolist()
    assert all(o in t for o, t in zip(out, top)), (out, top)
    assert lg[-3].argmax().item() == out[0]


def test_encoder_training_forward_matches_serving():
    from nv_genai_amd.models.encoder import EncoderModel
    from nv_genai_amd.training import functional as Fn

    m = EncoderModel(encoder_config("encoder-tiny"), "cpu", seed=3)
    seqs = [[101, 7, 8, 9, 102], [101, 11, 102]]
    ids = torch.tensor([t for s in seqs for t in s], dtype=torch.int32)
    pos = torch.tensor([p for s in seqs for p in range(len(s))], dtype=torch.int32)
    cu = torch.tensor([0, 5, 8], dtype=torch.int32)
    ref = m.forward(ids, pos, cu, 5)
    pad = torch.zeros(2, 5, dtype=torch.long)
    mask = torch.zeros(2, 5, dtype=torch.long)
    for b, s in enumerate(seqs):
        pad[b, : len(s)] = torch.tensor(s)
        mask[b, : len(s)] = 1
    got = Fn.encoder_embed(m, pad, mask)
    assert torch.allclose(got, ref.float(), atol=3e-2), (got - ref).abs().max()


def test_lora_identity_merge_and_save(tmp_path):
    from nv_genai_amd.training import functional as Fn
    from nv_genai_amd.training.lora import LoRA, LoRAConfig

    m = _llama()
    ids = torch.randint(0, 30000, (2, 12))
    base = Fn.llama_hidden(m, ids)
    ad = LoRA(m, LoRAConfig(r=4, alpha=8, targets=("qkv", "down")))
    assert torch.equal(Fn.llama_hidden(m, ids, linear=ad.linear), base)      # B = 0 at init
    with torch.no_grad():
        for b in ad.B.values():
            b.normal_(0, 0.05)
    with_ad = Fn.llama_hidden(m, ids, linear=ad.linear)
    ad.save(str(tmp_path / "ad"))
    ad.merge()
    merged = Fn.llama_hidden(m, ids)
    assert (merged.float() - with_ad.float()).abs().max() < 0.1
    ad.unmerge()
    ad2 = LoRA.load(m, str(tmp_path / "ad"))
    assert torch.equal(Fn.llama_hidden(m, ids, linear=ad2.linear), with_ad)


@pytest.mark.parametrize("lora", [True, False])
def test_sft_loss_decreases(lora):
    from nv_genai_amd.training.lora import LoRAConfig
    from nv_genai_amd.training.sft import TrainConfig, sft_trainer

    m = _llama()
    cfg = TrainConfig(lr=1e-2 if lora else 1e-3, warmup_steps=2, max_steps=12, micro_batch=4, global_batch=8,
                      max_seq_len=64, log_every=0)
    tr, _ = sft_trainer(m, CharTok(), DATA, cfg, LoRAConfig(r=8, alpha=16, targets=("qkv", "o", "gate_up", "down")) if lora else None)
    hist = tr.fit()
    # (the frozen random-init LM head bounds how far a LoRA-only run can push the loss)
    assert min(hist[-4:]) < hist[0] * 0.85, hist


def test_checkpoint_resume_is_step_exact(tmp_path):
    from nv_genai_amd.training.lora import LoRAConfig
    from nv_genai_amd.training.sft import TrainConfig, sft_trainer

    cfg = TrainConfig(lr=3e-3, warmup_steps=1, max_steps=6, micro_batch=2, global_batch=4, max_seq_len=64,
                      log_every=0)
    lc = LoRAConfig(r=4, alpha=8)
    a, _ = sft_trainer(_llama(), CharTok(), DATA, cfg, lc)
    full = a.fit(6)
    ck = str(tmp_path / "ck")
    b, _ = sft_trainer(_llama(), CharTok(), DATA, cfg, lc, ckpt_dir=ck)
    b.fit(3)
    b.save(ck)
    c, _ = sft_trainer(_llama(), CharTok(), DATA, cfg, lc, ckpt_dir=ck)
    assert c.resume(ck) and c.step == 3
    resumed = c.fit(3)
    assert resumed[:3] == full[:3]                       # history restored
    assert resumed[3:] == pytest.approx(full[3:], rel=1e-5)


def _dp_worker(rank, world, port, out):
    import torch.distributed as dist

    from nv_genai_amd.training.lora import LoRAConfig
    from nv_genai_amd.training.sft import TrainConfig, sft_trainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    cfg = TrainConfig(lr=3e-3, warmup_steps=1, max_steps=3, micro_batch=2, global_batch=4, max_seq_len=64,
                      log_every=0, bucket_mb=0.004)
    tr, ad = sft_trainer(_llama(), CharTok(), DATA, cfg, LoRAConfig(r=4, alpha=8, targets=("qkv", "o")))
    assert len(tr.sync.buckets) > 1
    hist = tr.fit(3)
    if rank == 0:
        torch.save({"hist": hist, "sd": ad.state_dict()}, out)
    dist.destroy_process_group()


def test_data_parallel_equals_single_process(tmp_path):
    from nv_genai_amd.training.lora import LoRAConfig
    from nv_genai_amd.training.sft import TrainConfig, sft_trainer

    out = str(tmp_path / "dp.pt")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_dp_worker, args=(2, port, out), nprocs=2, join=True)
    dp = torch.load(out, weights_only=True)
    torch.manual_seed(0)
    cfg = TrainConfig(lr=3e-3, warmup_steps=1, max_steps=3, micro_batch=2, global_batch=4, max_seq_len=64,
                      log_every=0)
    # one rank, two micro-batches of accumulation == two ranks x one micro-batch
    tr, ad = sft_trainer(_llama(), CharTok(), DATA, cfg, LoRAConfig(r=4, alpha=8, targets=("qkv", "o")))
    hist = tr.fit(3)
    assert dp["hist"] == pytest.approx(hist, rel=1e-4)
    for k, v in ad.state_dict().items():
        assert torch.allclose(dp["sd"][k], v, atol=1e-5), k


def test_hard_negative_mining_semantics():
    import numpy as np

    from nv_genai_amd.training.hard_negatives import mine_hard_negatives

    g = torch.Generator().manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(37, 16, generator=g), dim=1)
    p = torch.nn.functional.normalize(torch.randn(200, 16, generator=g), dim=1)
    pos = [[i, (i * 7) % 200] for i in range(37)]
    got = mine_hard_negatives(q, p, pos, margin=0.95, num_negs=5, block=8)
    s = (q @ p.t()).numpy()
    for i in range(37):
        row = s[i].copy()
        thr = min(row[j] for j in pos[i]) * 0.95
        row[pos[i]] = -np.inf
        row[row > thr] = -np.inf
        order = [int(j) for j in np.argsort(-row) if np.isfinite(row[j])][:5]
        assert got[i] == order


def test_retrieval_metrics():
    from nv_genai_amd.training.retrieval_eval import evaluate

    qrels = {"q1": {"a": 1, "b": 1}, "q2": {"c": 2}}
    res = {"q1": {"a": 0.9, "x": 0.8, "b": 0.7}, "q2": {"y": 0.5, "c": 0.4}}
    ndcg, mp, rec, prec = evaluate(qrels, res, (1, 3))
    assert rec["Recall@1"] == 0.25 and rec["Recall@3"] == 1.0
    assert prec["P@1"] == 0.5
    assert mp["MAP@3"] == round(((1 + 2 / 3) / 2 + 0.5) / 2, 5)
    import math
    n1 = (1 + 1 / math.log2(4)) / (1 + 1 / math.log2(3))
    n2 = (2 / math.log2(3)) / 2
    assert abs(ndcg["NDCG@3"] - (n1 + n2) / 2) < 1e-4


def test_embedding_finetune_improves_recall():
    from nv_genai_amd.engine.embed_engine import EmbeddingEngine
    from nv_genai_amd.training import functional as Fn
    from nv_genai_amd.training.embed_finetune import embed_trainer
    from nv_genai_amd.training.hard_negatives import build_training_records, mine_hard_negatives
    from nv_genai_amd.training.retrieval_eval import dense_retrieve, evaluate
    from nv_genai_amd.training.sft import TrainConfig
    from nv_genai_amd.utils.synthetic import TextGen

    gen = TextGen(seed=5)
    passages = [gen.sentence(10, 14) for _ in range(48)]
    queries = [" ".join(p.split()[2:6]) for p in passages]         # a fragment of its passage
    eng = EmbeddingEngine("encoder-tiny", device="cpu", seed=2)

    def recall():
        q = eng.embed(queries, "query")
        p = eng.embed(passages, "passage")
        res = dense_retrieve(q, p, [str(i) for i in range(48)], [str(i) for i in range(48)], k=5)
        return evaluate({str(i): {str(i): 1} for i in range(48)}, res, (1, 5))[2]["Recall@5"]

    before = recall()
    negs = mine_hard_negatives(eng.embed(queries, "query"), eng.embed(passages, "passage"),
                               [[i] for i in range(48)], margin=0.99, num_negs=4)
    recs = build_training_records(queries, passages, [[i] for i in range(48)], negs)
    cfg = TrainConfig(lr=2e-4, warmup_steps=2, max_steps=24, micro_batch=8, global_batch=8, max_seq_len=64,
                      log_every=0)
    tr, params = embed_trainer(eng, recs, cfg, hard_negatives=2)
    hist = tr.fit()
    Fn.write_back(eng.model, params, "encoder")
    after = recall()
    assert hist[-1] < hist[0] and after > before, (before, after, hist[0], hist[-1])


def test_pretrain_packing_loss_and_serving_handoff(tmp_path):
    """SLM pretraining (training/pretrain.py): packed windows, loss falls from a from-scratch
    init, the weights written back are served by the engine, and the SFT trainer takes over."""
    from nv_genai_amd.engine.llm_engine import EngineConfig, LLMEngine, SamplingParams
    from nv_genai_amd.training import functional as Fn
    from nv_genai_amd.training.pretrain import init_slm, pack, pretrain_trainer
    from nv_genai_amd.training.sft import TrainConfig, sft_trainer

    w = pack([[5, 6, 7], [8, 9], [10]], 3, eos=2)
    assert w.tolist() == [[5, 6, 7, 2], [8, 9, 2, 10]]
    m = _llama()
    init_slm(m, seed=0)
    tok = CharTok()
    docs = [tok.encode(f"the cat sat on mat number {i % 7}. ") * 3 for i in range(64)]
    win = pack(docs, 32, 2)
    cfg = TrainConfig(lr=3e-3, warmup_steps=4, max_steps=60, micro_batch=8, global_batch=8, log_every=0,
                      betas=(0.9, 0.95), weight_decay=0.1)
    tr, params = pretrain_trainer(m, win, cfg, ckpt_dir=str(tmp_path / "ck"))
    hist = tr.fit()
    assert min(hist[-3:]) < 0.6 * hist[0], hist
    Fn.write_back(m, params, "llama")
    eng = LLMEngine(EngineConfig(model="llama-tiny", max_num_seqs=2, max_batched_tokens=256, max_model_len=256,
                                 kv_cache_blocks=8, use_graphs=False), device="cpu", model=m, model_cfg=m.cfg)
    prompt = tok.encode("the cat sat on mat number 3. the cat sat on ")
    out = eng.generate([prompt], SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))[0].output_ids
    assert out == tok.encode("mat")                      # the pretrained model learned the corpus
    st, _ = sft_trainer(m, tok, DATA, TrainConfig(lr=1e-3, warmup_steps=1, max_steps=2, micro_batch=4,
                                                  global_batch=4, max_seq_len=64, log_every=0))
    assert len(st.fit()) == 2


@pytest.mark.parametrize("name", ["mistral-tiny", "mixtral-tiny", "gemma-tiny", "starcoder2-tiny"])
def test_family_training_forward_matches_serving(name):
    """The differentiable forward of every decoder family (sliding window over a 130-token
    sequence, MoE routing, GeGLU / LayerNorm + biases) equals the serving forward."""
    from nv_genai_amd.models.llama import AttnMeta, LlamaModel
    from nv_genai_amd.training import functional as Fn

    cfg = llama_config(name)
    m = LlamaModel(cfg, "cpu", seed=2)
    m.allocate_kv_cache(4, 64)
    T = 130
    ids = torch.randint(3, 30000, (T,), generator=torch.Generator().manual_seed(4))
    meta = AttnMeta(kind="prefill", slots=torch.arange(T, dtype=torch.int32),
                    cu_q=torch.tensor([0, T], dtype=torch.int32), ctx_lens=torch.tensor([T], dtype=torch.int32),
                    block_tables=torch.arange(4, dtype=torch.int32).unsqueeze(0), max_q_len=T, max_ctx=T)
    serve = m.forward(ids.int(), torch.arange(T, dtype=torch.int32), meta).float()
    train = Fn.llama_hidden(m, ids.unsqueeze(0).long())[0].float()
    rel = ((train - serve).norm() / serve.norm()).item()
    assert rel < 0.03, (name, rel)


@pytest.mark.parametrize("name", ["gemma-tiny", "starcoder2-tiny"])
def test_family_lora_sft_loss_decreases(name):
    """LoRA SFT of the model-customisation notebooks' families (models/Gemma/lora.ipynb,
    models/Codegemma/lora.ipynb, models/StarCoder2/lora.ipynb)."""
    from nv_genai_amd.models.llama import LlamaModel
    from nv_genai_amd.training.lora import LoRAConfig
    from nv_genai_amd.training.sft import TrainConfig, sft_trainer

    m = LlamaModel(llama_config(name, max_position=256), "cpu", seed=0)
    cfg = TrainConfig(lr=1e-2, warmup_steps=2, max_steps=12, micro_batch=4, global_batch=8,
                      max_seq_len=64, log_every=0)
    tr, _ = sft_trainer(m, CharTok(), DATA, cfg, LoRAConfig(r=8, alpha=16, targets=("qkv", "o", "gate_up", "down")))
    hist = tr.fit()
    assert min(hist[-4:]) < hist[0] * 0.9, hist
