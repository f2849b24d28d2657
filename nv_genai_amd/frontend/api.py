"""RAG playground web app (frontend/frontend/api.py, pages/converse.py,
pages/kb.py). Gradio is not available here, so the two pages (Converse, Knowledge Base) are a
self-contained HTML/JS page served by FastAPI, talking to same-origin ``/api/*`` routes that
proxy the chain server through :class:`ChatClient` (trace context propagated).

Speech (the reference's Riva streaming ASR / TTS, frontend/frontend/asr_utils.py:106-155,
tts_utils.py:77-127): ``SPEECH_API_URI`` (or ``RIVA_API_URI``) names a speech server with the
OpenAI-style ``/v1/audio/transcriptions`` and ``/v1/audio/speech`` routes; the playground's
``/api/asr`` streams a recorded clip's transcripts back segment by segment (the reference's
running / finalized transcript updates) through :class:`dsp.asr.HTTPTranscriptionASR`, and
``/api/tts`` streams the answer's PCM16 chunks as they are synthesised (the reference's
``text_to_speech`` generator, with its 300-character segmentation) through
:class:`dsp.tts.HTTPSpeechTTS`. Without an endpoint both routes answer 501 and the UI hides
the speech controls.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse, JSONResponse, StreamingResponse

from ..chain_server.multipart import parse_multipart
from .chat_client import ChatClient

PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>RAG Playground (MI355X)</title>
<style>body{font-family:sans-serif;margin:0;background:#111;color:#eee}header{padding:12px 20px;background:#222}
nav button{margin-right:8px}main{padding:20px}#log{height:55vh;overflow:auto;border:1px solid #333;padding:10px;
white-space:pre-wrap}.u{color:#8cf}.a{color:#cfc}input[type=text]{width:70%}.hide{display:none}</style></head>
<body><header><b>RAG Playground</b> — model: <span id="model"></span>
<nav><button onclick="show('converse')">Converse</button><button onclick="show('kb')">Knowledge Base</button></nav></header>
<main><section id="converse"><div id="log"></div><p><input id="q" type="text" placeholder="Ask a question">
<button onclick="send()">Submit</button> <label><input id="kb" type="checkbox"> Use knowledge base</label>
<button onclick="document.getElementById('log').innerHTML=''">Clear</button></p>
<p id="speech" class="hide"><label>Transcribe audio <input id="audio" type="file" accept="audio/wav"
onchange="asr()"></label> <button onclick="speak()">Read answer aloud</button></p>
<details><summary>Show context</summary><pre id="ctx"></pre></details></section>
<section id="kb" class="hide"><p><input id="file" type="file" multiple> <button onclick="upload()">Upload</button></p>
<ul id="docs"></ul></section></main>
<script>
function show(id){for(const s of ['converse','kb'])document.getElementById(s).classList.toggle('hide',s!==id);if(id==='kb')docs();}
async function send(){const q=document.getElementById('q').value;if(!q)return;const kb=document.getElementById('kb').checked;
const log=document.getElementById('log');log.innerHTML+='<div class=u>'+q.replace(/</g,'&lt;')+'</div>';
const a=document.createElement('div');a.className='a';log.appendChild(a);
if(kb){const r=await fetch('/api/search',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({query:q})});
document.getElementById('ctx').textContent=JSON.stringify(await r.json(),null,1);}
const r=await fetch('/api/generate',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({query:q,use_knowledge_base:kb})});
const rd=r.body.getReader();const dec=new TextDecoder();let buf='';
for(;;){const {value,done}=await rd.read();if(done)break;buf+=dec.decode(value,{stream:true});let i;
while((i=buf.indexOf('\\n'))>=0){const line=buf.slice(0,i);buf=buf.slice(i+1);if(line)a.textContent+=JSON.parse(line).text;}log.scrollTop=log.scrollHeight;}}
async function docs(){const r=await fetch('/api/documents');const d=await r.json();const ul=document.getElementById('docs');ul.innerHTML='';
for(const f of d.documents){const li=document.createElement('li');li.textContent=f+' ';const b=document.createElement('button');b.textContent='delete';
b.onclick=async()=>{await fetch('/api/documents?filename='+encodeURIComponent(f),{method:'DELETE'});docs();};li.appendChild(b);ul.appendChild(li);}}
async function upload(){const fs=document.getElementById('file').files;for(const f of fs){const fd=new FormData();fd.append('file',f);
await fetch('/api/documents',{method:'POST',body:fd});}docs();}
async function asr(){const f=document.getElementById('audio').files[0];if(!f)return;
const r=await fetch('/api/asr',{method:'POST',body:await f.arrayBuffer(),headers:{'Content-Type':'audio/wav'}});
const q=document.getElementById('q');q.value='';for(const line of (await r.text()).split('\n'))if(line)q.value+=(q.value?' ':'')+JSON.parse(line).text;}
async function speak(){const as=document.querySelectorAll('#log .a');if(!as.length)return;
const r=await fetch('/api/tts?format=wav',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({text:as[as.length-1].textContent})});
new Audio(URL.createObjectURL(await r.blob())).play();}
fetch('/api/config').then(r=>r.json()).then(c=>{document.getElementById('model').textContent=c.model_name;
document.getElementById('speech').classList.toggle('hide',!c.speech);});
</script></body></html>"""


def speech_url() -> Optional[str]:
    return os.environ.get("SPEECH_API_URI") or os.environ.get("RIVA_API_URI") or None


def _pcm_of(body: bytes, rate: int):
    """(PCM16 bytes, sample rate) of an uploaded clip: a WAV file, or raw PCM16 at ``rate``."""
    import io
    import wave

    if body[:4] == b"RIFF":
        with wave.open(io.BytesIO(body)) as w:
            if w.getsampwidth() != 2 or w.getnchannels() != 1:
                raise ValueError("speech input must be mono 16-bit PCM")
            return w.readframes(w.getnframes()), w.getframerate()
    return body, rate


def create_frontend(client: ChatClient, asr=None, tts=None) -> FastAPI:
    """``asr`` / ``tts``: speech backends (``dsp.asr.ASRBackend`` with a ``rate``, and an object
    with ``synthesize(text, voice)`` yielding (rate, int16 array) chunks); by default built
    from ``SPEECH_API_URI`` / ``RIVA_API_URI`` when set."""
    app = FastAPI(title="RAG playground")
    app.state.client = client
    url = speech_url()
    if url and asr is None:
        from ..dsp.asr import HTTPTranscriptionASR

        asr = HTTPTranscriptionASR(url, model=os.environ.get("SPEECH_ASR_MODEL", "asr"),
                                   segment_s=float(os.environ.get("SPEECH_ASR_SEGMENT_S", "5")))
    if url and tts is None:
        from ..dsp.tts import HTTPSpeechTTS

        tts = HTTPSpeechTTS(url, model=os.environ.get("SPEECH_TTS_MODEL", "tts"),
                            voice=os.environ.get("SPEECH_TTS_VOICE", "default"))

    @app.get("/", response_class=HTMLResponse)
    @app.get("/content/converse", response_class=HTMLResponse)
    @app.get("/content/kb", response_class=HTMLResponse)
    def page():
        return PAGE

    @app.get("/api/config")
    def config():
        return {"model_name": client.model_name, "server_url": client.server_url,
                "speech": asr is not None and tts is not None}

    @app.post("/api/generate")
    async def generate(request: Request):
        body = await request.json()

        def lines():
            for chunk in client.predict(body.get("query", ""), bool(body.get("use_knowledge_base")),
                                        int(body.get("num_tokens", 1024))):
                if chunk:
                    yield json.dumps({"text": chunk}) + "\n"

        return StreamingResponse(lines(), media_type="application/x-ndjson")

    @app.post("/api/search")
    async def search(request: Request):
        body = await request.json()
        return client.search(body.get("query", ""), int(body.get("top_k", 4)))

    @app.get("/api/documents")
    def documents():
        return {"documents": client.get_uploaded_documents()}

    @app.delete("/api/documents")
    def delete(filename: str):
        return {"message": client.delete_documents(filename)}

    @app.post("/api/documents")
    async def upload(request: Request):
        parts = parse_multipart(await request.body(), request.headers.get("content-type", ""))
        name, data = parts.get("file", (None, b""))
        if not name:
            return JSONResponse({"message": "No files provided"})
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, os.path.basename(name))
            with open(p, "wb") as f:
                f.write(data)
            try:
                client.upload_documents([p])
            except ValueError as e:
                return JSONResponse({"message": str(e)}, status_code=500)
        return {"message": "File uploaded successfully"}

    @app.post("/api/asr")
    async def transcribe(request: Request, rate: int = 16000, chunk_ms: int = 100):
        """Recorded clip (WAV, or raw PCM16 at ``rate``) -> NDJSON transcripts, one line per
        recognised segment ({"text", "final"}), streamed as the recogniser produces them."""
        if asr is None:
            return JSONResponse({"message": "speech requires a speech endpoint (SPEECH_API_URI)"},
                                status_code=501)
        import wave

        try:
            pcm, sr = _pcm_of(await request.body(), rate)
        except (ValueError, EOFError, wave.Error) as e:   # malformed RIFF / PCM: the client's fault
            return JSONResponse({"message": str(e)}, status_code=400)
        if getattr(asr, "rate", sr) != sr:
            return JSONResponse({"message": f"the recogniser takes {asr.rate} Hz audio, got {sr} Hz"},
                                status_code=400)
        step = max(2, int(sr * chunk_ms / 1000) * 2)
        chunks = (pcm[i:i + step] for i in range(0, len(pcm), step))

        def lines():
            for text, final in asr.stream(chunks):
                yield json.dumps({"text": text, "final": bool(final)}) + "\n"

        return StreamingResponse(lines(), media_type="application/x-ndjson")

    @app.post("/api/tts")
    async def speak(request: Request, format: str = "pcm"):
        """{"text", "voice"?} -> the synthesised answer: raw PCM16 chunks streamed as they
        arrive (``X-Sample-Rate`` header; first audio before the whole answer is rendered),
        or one WAV file with ``?format=wav``."""
        if tts is None:
            return JSONResponse({"message": "speech requires a speech endpoint (SPEECH_API_URI)"},
                                status_code=501)
        body = await request.json()
        text = str(body.get("text", "")).strip()
        if not text:
            return JSONResponse({"message": "no text to synthesise"}, status_code=400)
        from starlette.concurrency import run_in_threadpool

        # the speech client does blocking HTTP: its calls run in the threadpool, never on the
        # event loop (a long answer would otherwise stall every other route)
        gen = tts.synthesize(text, body.get("voice"))
        first = await run_in_threadpool(next, gen, None)
        if first is None:
            return JSONResponse({"message": "the speech server returned no audio"}, status_code=502)
        rate = int(first[0])
        if format == "wav":
            def render() -> bytes:
                import io
                import wave

                buf = io.BytesIO()
                with wave.open(buf, "wb") as w:
                    w.setnchannels(1)
                    w.setsampwidth(2)
                    w.setframerate(rate)
                    w.writeframes(first[1].astype("<i2").tobytes())
                    for _, pcm in gen:
                        w.writeframes(pcm.astype("<i2").tobytes())
                return buf.getvalue()

            return StreamingResponse(iter([await run_in_threadpool(render)]), media_type="audio/wav")

        def chunks():
            yield first[1].astype("<i2").tobytes()
            for _, pcm in gen:
                if len(pcm):
                    yield pcm.astype("<i2").tobytes()

        return StreamingResponse(chunks(), media_type=f"audio/L16;rate={rate}",
                                 headers={"X-Sample-Rate": str(rate)})

    return app
