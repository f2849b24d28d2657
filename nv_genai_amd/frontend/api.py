"""RAG playground web app (frontend/frontend/api.py, pages/converse.py,
pages/kb.py). Gradio is not available here, so the two pages (Converse, Knowledge Base) are a
self-contained HTML/JS page served by FastAPI, talking to same-origin ``/api/*`` routes that
proxy the chain server through :class:`ChatClient` (trace context propagated).

Speech (Riva streaming ASR / TTS, asr_utils.py / tts_utils.py) needs a Riva endpoint: the
routes answer 501 unless ``RIVA_API_URI`` is configured, and the UI hides the mic/speaker.
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
fetch('/api/config').then(r=>r.json()).then(c=>document.getElementById('model').textContent=c.model_name);
</script></body></html>"""


def create_frontend(client: ChatClient) -> FastAPI:
    app = FastAPI(title="RAG playground")
    app.state.client = client

    @app.get("/", response_class=HTMLResponse)
    @app.get("/content/converse", response_class=HTMLResponse)
    @app.get("/content/kb", response_class=HTMLResponse)
    def page():
        return PAGE

    @app.get("/api/config")
    def config():
        return {"model_name": client.model_name, "server_url": client.server_url,
                "speech": bool(os.environ.get("RIVA_API_URI"))}

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
    @app.post("/api/tts")
    def speech():
        if not os.environ.get("RIVA_API_URI"):
            return JSONResponse({"message": "speech requires a Riva endpoint (RIVA_API_URI)"}, status_code=501)
        return JSONResponse({"message": "Riva client library not installed on this image"}, status_code=501)

    return app
