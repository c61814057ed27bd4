"""Streamlit dashboard (drop-in for the reference's app_ui.py, R-21..R-25).

Tabs: single-dialogue analysis (prediction badge + confidence + LLM explanation), batch CSV
prediction (one GPU launch for the whole file, downloadable CSV) and real-time Kafka monitoring
(batched, commit-after-produce). All logic lives in
``fraud_detection_spark_kafka_llm_amd.serve.ui_logic``; this file is layout only.

    streamlit run app_ui.py          (MODEL_PATH env var overrides dialogue_classification_model)
"""
import os

import pandas as pd
import streamlit as st

st.set_page_config(page_title="Dialogue Classifier", layout="wide")

from fraud_detection_spark_kafka_llm_amd.serve import ui_logic  # noqa: E402
from fraud_detection_spark_kafka_llm_amd.utils.config import load_dotenv  # noqa: E402
from utils.st_functions import load_css, styled_badge  # noqa: E402

load_css("public/main.css")
load_dotenv()
from utils.agent_api import DeepSeekClassificationAgent  # noqa: E402  (validates DEEPSEEK_API_KEY)
from utils.kafka_utils import get_kafka_consumer, get_kafka_producer  # noqa: E402

MODEL_PATH = os.getenv("MODEL_PATH", "dialogue_classification_model")


@st.cache_resource
def load_agent():
    return DeepSeekClassificationAgent(model_path=MODEL_PATH)


agent = load_agent()

st.title("📞 Customer Dialogue Classifier")
st.markdown("AI-powered tool for identifying potential fraud in customer dialogues — MI355X-native engine.")

with st.sidebar:
    st.header("⚙️ Settings")
    temperature = st.slider("AI Creativity", 0.1, 1.0, 0.7)
    show_confidence = st.checkbox("Show confidence scores", True)
    show_history = st.checkbox("Show historical insights", False)
    st.divider()
    st.header("📂 Upload Historical Data")
    uploaded = st.file_uploader("Upload CSV with historical dialogues", type=["csv"],
                                help="Must contain a 'dialogue' column")
    uploaded_df = None
    if uploaded:
        try:
            uploaded_df = pd.read_csv(uploaded)
            if "dialogue" not in uploaded_df.columns:
                st.error("CSV must contain a 'dialogue' column.")
                uploaded_df = None
            else:
                agent.historical_data = uploaded_df
                st.success(f"Loaded {len(uploaded_df)} records.")
                st.dataframe(uploaded_df.head(), use_container_width=True)
        except Exception as e:
            st.error(f"Error loading file: {e}")

tab1, tab2, tab3 = st.tabs(["🔍 Single Dialogue Analysis", "📊 Batch Prediction (CSV)", "📡 Real-time Monitoring"])

with tab1:
    user_input = st.text_area("Enter a customer service dialogue:", height=200, placeholder="Paste your dialogue here...")
    if st.button("Analyze"):
        with st.spinner("Analyzing..."):
            try:
                res = ui_logic.analyze_single(agent, user_input, temperature, with_history=show_history)
                st.subheader("🔎 Prediction Result")
                cols = st.columns(2)
                cols[0].text("Prediction")
                text, color = ui_logic.badge_for(res["prediction"])
                cols[0].markdown(styled_badge(text, color), unsafe_allow_html=True)
                if show_confidence and res["confidence"] is not None:
                    cols[1].metric("Confidence", f"{res['confidence'] * 100:.0f}%")
                if res["error"]:
                    st.error(res["error"])
                else:
                    with st.expander("🧠 AI Explanation", expanded=True):
                        st.write(res["analysis"])
                    if show_history and res["historical_insight"]:
                        with st.expander("📚 Historical Context"):
                            st.write(res["historical_insight"])
            except Exception as e:
                st.error(f"An error occurred: {e}")

with tab2:
    st.write("Upload a CSV with a `dialogue` column to classify multiple entries.")
    if uploaded_df is not None:
        if st.button("Predict Labels for Uploaded CSV"):
            with st.spinner("Predicting..."):
                try:
                    table, csv = ui_logic.predict_dataframe(agent, uploaded_df)
                    st.success("Batch classification complete.")
                    st.dataframe(table, use_container_width=True)
                    st.download_button("📥 Download Results as CSV", data=csv, file_name="predicted_dialogues.csv",
                                       mime="text/csv")
                except Exception as e:
                    st.error(f"Error during prediction: {e}")
    else:
        st.info("Upload a CSV file in the sidebar to enable batch classification.")

with tab3:
    st.header("Real-time Dialogue Monitoring")
    if "kafka_running" not in st.session_state:
        st.session_state.kafka_running = False
        st.session_state.monitor = None
    c1, c2 = st.columns(2)
    if c1.button("Start Monitoring") and not st.session_state.kafka_running:
        st.session_state.kafka_running = True
        st.rerun()
    if c2.button("Stop Monitoring") and st.session_state.kafka_running:
        st.session_state.kafka_running = False
        st.rerun()
    if st.session_state.kafka_running:
        status, board = st.empty(), st.empty()
        consumer, producer = get_kafka_consumer(), get_kafka_producer()
        mon = ui_logic.KafkaMonitor(agent, consumer, producer, os.getenv("KAFKA_OUTPUT_TOPIC"),
                                    temperature=temperature)
        try:
            while st.session_state.kafka_running:
                if mon.step(timeout=1.0) == 0:
                    continue
                status.success(f"Processed {len(mon.messages)} messages ({len(mon.errors)} skipped)")
                board.markdown("".join(ui_logic.render_message_card(m) for m in mon.last(5)), unsafe_allow_html=True)
        finally:
            consumer.close()
