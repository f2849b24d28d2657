"""FM-radio front end for streaming ASR RAG.

``design``  — FIR design (Hamming-windowed sinc ``firwin``) and the polyphase decimator
              taps/alignment of ``resample_poly``;
``sdr``     — the burst pipeline on the GPU (low-pass → FM demod → decimate → gain → PCM16)
              and the UDP I/Q receiver;
``replay``  — WAV → FM-modulated I/Q → UDP packets (the reference's file-replay tool);
``asr``     — ASR backends + the transcript exporter that feeds the FM-ASR chain server.
"""
