"""Streamlit helpers (R-20): CSS injection and a pill-shaped status badge."""
from __future__ import annotations

import html

_BOOTSTRAP = ('<link rel="stylesheet" href="https://maxcdn.bootstrapcdn.com/bootstrap/4.0.0/css/bootstrap.min.css" '
              'crossorigin="anonymous">')


def css_block(css_text: str) -> str:
    return f"<style>{css_text}</style>"


def load_css(file_css: str) -> None:
    """Inject a stylesheet into the page (adds Bootstrap when the file is ``style.css``)."""
    import streamlit as st

    with open(file_css, encoding="utf-8") as fh:
        st.markdown(css_block(fh.read()), unsafe_allow_html=True)
    if file_css == "style.css":
        st.markdown(_BOOTSTRAP, unsafe_allow_html=True)


def styled_badge(text: str, bg_color: str) -> str:
    """HTML for a rounded, bold label with white text on ``bg_color``."""
    return (f'<span style="background-color:{html.escape(bg_color, quote=True)};color:white;'
            f'padding:4px 10px;border-radius:12px;font-weight:bold;font-size:0.9rem;">{html.escape(text)}</span>')
