"""Local LLM chat UI (drop-in for the reference's deepseek_chat_ui.py, R-26).

Streamlit chat against an OpenAI-compatible server (LM Studio by default). Uses the framework's
``ChatClient`` (retrying, no ``openai`` package needed). ``FDX_LLM_BASE_URL`` / ``FDX_LLM_MODEL``
override the endpoint; ``python -m fraud_detection_spark_kafka_llm_amd.serve.llm_stub`` serves an
offline stand-in.
"""
import os

import streamlit as st

from fraud_detection_spark_kafka_llm_amd.serve.llm import ChatClient

BASE_URL = os.getenv("FDX_LLM_BASE_URL", "http://192.168.56.1:1234/v1")
MODEL_NAME = os.getenv("FDX_LLM_MODEL", "deepseek-r1-0528-qwen3-8b")
client = ChatClient(api_key="not-needed", model=MODEL_NAME, base_url=BASE_URL, timeout=120)

st.set_page_config(page_title="DeepSeek Chat", layout="centered")
with st.sidebar:
    st.title("🤖 DeepSeek Chat (Local)")
    st.markdown(f"Connected to an OpenAI-compatible server at `{BASE_URL}`.")
    st.markdown("---")
    temperature = st.slider("Response Creativity (Temperature)", 0.0, 1.5, 0.7, 0.05)

st.title("💬 Chat with DeepSeek (Local)")
if "messages" not in st.session_state:
    st.session_state.messages = [{"role": "system", "content": "You are a helpful assistant."}]
for m in st.session_state.messages:
    if m["role"] != "system":
        with st.chat_message(m["role"]):
            st.markdown(m["content"])

prompt = st.chat_input("Ask me anything...")
if prompt:
    st.session_state.messages.append({"role": "user", "content": prompt})
    with st.chat_message("user"):
        st.markdown(prompt)
    with st.chat_message("assistant"):
        with st.spinner("Thinking..."):
            try:
                reply = client.chat(st.session_state.messages, temperature=temperature, max_tokens=2048)
            except Exception as e:
                reply = f"⚠️ Error: {e}"
        st.markdown(reply)
        st.session_state.messages.append({"role": "assistant", "content": reply})
