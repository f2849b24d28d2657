"""Application configuration schema (``APP_*`` parity with the reference's AppConfig,
RetrievalAugmentedGeneration/common/configuration.py:21-258), plus the sections this
framework adds for its own engines (``APP_ENGINE_*``, ``APP_INDEX_*``).

Compatibility notes:
* ``vector_store.name`` accepts the reference's ``milvus`` / ``pgvector`` / ``faiss`` values;
  all of them are served by the in-HBM index of this framework (``flat`` or ``ivf_flat``),
  with Milvus' ``GPU_IVF_FLAT`` nlist/nprobe knobs honoured when ``index.type=ivf_flat``.
* ``llm.model_engine``: ``local`` runs the model in-process on this GPU;
  ``nvidia-ai-endpoints`` / ``openai`` talk the OpenAI/NIM HTTP protocol to ``server_url``
  (e.g. this framework's model server), exactly like ChatNVIDIA(base_url=...).
"""
from __future__ import annotations

from .config_wizard import ConfigWizard, configclass, configfield


@configclass
class VectorStoreConfig(ConfigWizard):
    name: str = configfield("name", default="milvus", help_txt="The name of vector store")
    url: str = configfield("url", default="http://milvus:19530",
                           help_txt="The host of the machine running Vector Store DB")
    nlist: int = configfield("nlist", default=64, help_txt="Number of cluster units")
    nprobe: int = configfield("nprobe", default=16, help_txt="Number of units to query")


@configclass
class LLMConfig(ConfigWizard):
    server_url: str = configfield("server_url", default="",
                                  help_txt="The location of the server hosting the llm model.")
    model_name: str = configfield("model_name", default="ensemble",
                                  help_txt="The name of the hosted model.")
    model_engine: str = configfield(
        "model_engine", default="nvidia-ai-endpoints",
        help_txt="Server type of the hosted model: local | nvidia-ai-endpoints | openai")
    model_name_pandas_ai: str = configfield(
        "model_name_pandas_ai", default="ai-mixtral-8x7b-instruct",
        help_txt="The name of the model used by the structured-data (pandas) agent")


@configclass
class TextSplitterConfig(ConfigWizard):
    model_name: str = configfield(
        "model_name", default="Snowflake/snowflake-arctic-embed-l",
        help_txt="Tokenizer model used by the token text splitter.")
    chunk_size: int = configfield("chunk_size", default=510, help_txt="Chunk size for text splitting.")
    chunk_overlap: int = configfield("chunk_overlap", default=200,
                                     help_txt="Overlapping text length for splitting.")


@configclass
class EmbeddingConfig(ConfigWizard):
    model_name: str = configfield("model_name", default="snowflake/arctic-embed-l",
                                  help_txt="The name of the embedding model.")
    model_engine: str = configfield(
        "model_engine", default="nvidia-ai-endpoints",
        help_txt="Server type of the embedding model: local | nvidia-ai-endpoints | openai")
    dimensions: int = configfield("dimensions", default=1024,
                                  help_txt="Embedding dimensions (vector index width).")
    server_url: str = configfield("server_url", default="",
                                  help_txt="The url of the server hosting the embedding model")


@configclass
class RetrieverConfig(ConfigWizard):
    top_k: int = configfield("top_k", default=4, help_txt="Number of relevant results to retrieve")
    score_threshold: float = configfield(
        "score_threshold", default=0.25,
        help_txt="The minimum confidence score for the retrieved values to be considered")
    nr_url: str = configfield("nr_url", default="http://retrieval-ms:8000",
                              help_txt="The retriever microservice url")
    nr_pipeline: str = configfield("nr_pipeline", default="ranked_hybrid",
                                   help_txt="Retriever pipeline: ranked_hybrid | hybrid | dense")


@configclass
class PromptsConfig(ConfigWizard):
    chat_template: str = configfield(
        "chat_template",
        default=("You are a helpful, respectful and honest assistant."
                 "Always answer as helpfully as possible, while being safe."
                 "Please ensure that your responses are positive in nature."),
        help_txt="Prompt template for chat.")
    rag_template: str = configfield(
        "rag_template",
        default=("<s>[INST] <<SYS>>"
                 "Use the following context to answer the user's question. If you don't know the answer,"
                 "just say that you don't know, don't try to make up an answer."
                 "<</SYS>>"
                 "<s>[INST] Context: {context_str} Question: {query_str} Only return the helpful"
                 " answer below and nothing else. Helpful answer:[/INST]"),
        help_txt="Prompt template for rag.")
    multi_turn_rag_template: str = configfield(
        "multi_turn_rag_template",
        default=("You are a document chatbot. Help the user as they ask questions about documents."
                 " User message just asked: {input}\n\n"
                 " For this, we have retrieved the following potentially-useful info: "
                 " Conversation History Retrieved:\n{history}\n\n"
                 " Document Retrieved:\n{context}\n\n"
                 " Answer only from retrieved data. Make your response conversational."),
        help_txt="Prompt template for multi-turn rag.")


@configclass
class EngineConfigSection(ConfigWizard):
    """In-process engines on this node (model_engine=local)."""

    llm_preset: str = configfield("llm_preset", default="llama3-8b",
                                  help_txt="LLM architecture preset (llama3-8b | llama3-70b | llama-small | llama-tiny)")
    embed_preset: str = configfield("embed_preset", default="arctic-embed-l",
                                    help_txt="Encoder preset (arctic-embed-l | e5-large-v2 | all-minilm-l6-v2 | encoder-tiny)")
    rerank_preset: str = configfield("rerank_preset", default="",
                                     help_txt="Cross-encoder reranker preset ('' = disabled)")
    weights_dir: str = configfield("weights_dir", default="",
                                   help_txt="Directory of safetensors weights ('' = random init)")
    tp_size: int = configfield("tp_size", default=1, help_txt="Tensor-parallel degree of the LLM")
    pp_size: int = configfield("pp_size", default=1, help_txt="Pipeline stages of the LLM (layer split)")
    sequence_parallel: bool = configfield("sequence_parallel", default=False,
                                          help_txt="Sequence-parallel TP prefill (reduce-scatter/all-gather)")
    kv_cache_fraction: float = configfield("kv_cache_fraction", default=0.3,
                                           help_txt="Fraction of free HBM given to the paged KV cache")
    max_num_seqs: int = configfield("max_num_seqs", default=256, help_txt="Max concurrent sequences")
    max_model_len: int = configfield("max_model_len", default=8192, help_txt="Max prompt + output tokens")
    max_batched_tokens: int = configfield("max_batched_tokens", default=16384,
                                          help_txt="Token budget of one prefill step")
    device: str = configfield("device", default="", help_txt="Device ('' = cuda if available)")
    kv_cache_dtype: str = configfield("kv_cache_dtype", default="auto",
                                      help_txt="auto | fp8 (e4m3fn KV pages: twice the cached tokens)")
    fp8: bool = configfield("fp8", default=False, help_txt="W8A8 FP8 projections of the LLM")


@configclass
class IndexConfig(ConfigWizard):
    type: str = configfield("type", default="flat", help_txt="flat | ivf_flat | hnsw")
    metric: str = configfield("metric", default="cosine", help_txt="cosine | ip | l2")
    persist_dir: str = configfield("persist_dir", default="",
                                   help_txt="Directory for index snapshots ('' = in-memory only)")
    shards: int = configfield("shards", default=1,
                              help_txt="Shard the index across this many ranks (RCCL merge)")
    synthetic_docs: int = configfield("synthetic_docs", default=0,
                                      help_txt="Fill the default collection with this many synthetic chunks and "
                                               "random unit vectors (benchmarks; 0 = off)")


@configclass
class AppConfig(ConfigWizard):
    vector_store: VectorStoreConfig = configfield(
        "vector_store", env=False, default=VectorStoreConfig(),
        help_txt="The configuration of the vector db connection.")
    llm: LLMConfig = configfield("llm", env=False, default=LLMConfig(),
                                 help_txt="The configuration for the server hosting the Large Language Models.")
    text_splitter: TextSplitterConfig = configfield(
        "text_splitter", env=False, default=TextSplitterConfig(),
        help_txt="The configuration for text splitter.")
    embeddings: EmbeddingConfig = configfield("embeddings", env=False, default=EmbeddingConfig(),
                                              help_txt="The configuration of embedding model.")
    retriever: RetrieverConfig = configfield("retriever", env=False, default=RetrieverConfig(),
                                             help_txt="The configuration of the retriever pipeline.")
    prompts: PromptsConfig = configfield("prompts", env=False, default=PromptsConfig(),
                                         help_txt="Prompt templates for chat and rag.")
    engine: EngineConfigSection = configfield("engine", env=False, default=EngineConfigSection(),
                                              help_txt="In-process engine settings (MI355X).")
    index: IndexConfig = configfield("index", env=False, default=IndexConfig(),
                                     help_txt="Vector index settings (MI355X in-HBM index).")
