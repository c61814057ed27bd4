"""Classification agent (R-16): saved Spark-layout pipeline -> fused gfx950 scorer -> LLM explanation.

Same public surface as the reference's ``DeepSeekClassificationAgent``
(/root/reference/utils/agent_api.py:124-208): ``model``, ``analyzer``, ``historical_data``,
``preprocess_text``, ``predict_and_get_label``, ``classify_and_explain``,
``find_similar_historical_cases``. Differences:

* one fused kernel launch per call (the reference runs two Spark jobs per prediction);
* ``predict_batch`` scores a whole list in one launch (batch CSV tab, streaming);
* ``classify_and_explain`` can reuse an existing prediction, and passes ``temperature`` through;
* ``find_similar_historical_cases`` ranks historical dialogues by cosine similarity of their
  TF-IDF vectors (the reference returns the first ``n`` rows as a placeholder).

``confidence`` keeps the reference's meaning: P(class 1 = fraud), whatever the prediction.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ..ml import Frame, PipelineModel, TextColumn
from ..ml.fused import FusedPipeline
from ..ops.sparse import score_csr
from ..ops.text import LinearScorer, PackedText, featurize_score
from ..utils.config import default_device
from ..utils.logging import get_logger
from .llm import Analyzer, make_llm

log = get_logger("agent")


class ClassificationAgent:
    def __init__(self, model_path: str, historical_data_path: Optional[str] = None, llm=None, device=None,
                 analyzer: Optional[Analyzer] = None):
        self.device = torch.device(device) if device is not None else default_device()
        self.model = PipelineModel.load(model_path)
        self.fused: FusedPipeline = self.model.compile(self.device)
        self.analyzer = analyzer or Analyzer(llm if llm is not None else make_llm())
        self._historical: Optional[Frame] = None
        self._hist_index = None
        if historical_data_path:
            self.historical_data = Frame.read_csv(historical_data_path)

    # ------------------------------------------------------------------ historical data
    @property
    def historical_data(self) -> Optional[Frame]:
        return self._historical

    @historical_data.setter
    def historical_data(self, frame) -> None:
        if frame is not None and not isinstance(frame, Frame):
            frame = Frame.from_pandas(frame)
        self._historical = frame
        self._hist_index = None

    # ------------------------------------------------------------------ inference
    def preprocess_text(self, text: str) -> Frame:
        raw = TextColumn([text])
        return Frame({"dialogue": raw, "clean_text": TextColumn.cleaned_from(raw)})

    def predict_batch(self, texts: Sequence[str]) -> list:
        if not len(texts):
            return []
        pred, prob, _ = self.fused.predict([t if t is not None else "" for t in texts], clean=True)
        pred = pred.cpu().numpy()
        p1 = prob[:, 1].cpu().numpy()
        return [{"prediction": float(a), "confidence": float(b)} for a, b in zip(pred, p1)]

    def predict_and_get_label(self, text: str) -> dict:
        try:
            return self.predict_batch([text])[0]
        except Exception as e:  # keep the reference's contract: prediction even if confidence fails
            log.error("prediction failed: %s", e)
            raise

    def find_similar_historical_cases(self, dialogue: str, n: int = 3):
        hd = self._historical
        if hd is None or hd.count() == 0 or "dialogue" not in hd:
            return None
        if self._hist_index is None:
            texts = [s or "" for s in (hd.column("dialogue").strings if isinstance(hd.column("dialogue"), TextColumn)
                                       else list(hd.column("dialogue")))]
            vc = self._features(texts)
            ip, ix, v = vc.csr()
            norms = torch.zeros(len(texts), dtype=torch.float64, device=v.device)
            row = torch.repeat_interleave(torch.arange(len(texts), device=v.device), ip[1:] - ip[:-1])
            norms.index_add_(0, row, v.double() * v.double())
            self._hist_index = (vc, torch.sqrt(norms))
        vc, norms = self._hist_index
        q = self._features([dialogue])
        qi, qx, qv = q.csr()
        w = np.zeros(q.size)
        w[qx.cpu().numpy()] = qv.cpu().double().numpy()
        qn = float(np.linalg.norm(w))
        if qn == 0:
            return hd.limit(n).collect()
        sims = score_csr(vc, LinearScorer(w, 0.0))[:, 0] / torch.clamp(norms * qn, min=1e-12)
        top = torch.argsort(sims, descending=True, stable=True)[:n].cpu().numpy()
        return hd.take_rows(top).collect()

    def _features(self, texts):
        fp = self.fused
        idf = fp.idf.idf_tensor(self.device) if fp.idf is not None else None
        res = featurize_score(PackedText.from_strings(texts), fp.spec(True), idf=idf, want_csr=True, device=self.device)
        ip, ix, v = res.csr()
        from ..ml.linalg import VectorColumn

        return VectorColumn(fp.dim, ip, ix, v.to(torch.float64))

    def classify_and_explain(self, dialogue: str, temperature: float = 0.7, prediction: Optional[dict] = None,
                             with_history: bool = True) -> dict:
        res = prediction or self.predict_and_get_label(dialogue)
        analysis = self.analyzer.analyze_prediction(dialogue, res["prediction"], res["confidence"], temperature)
        insight = None
        if with_history and self._historical is not None:
            cases = self.find_similar_historical_cases(dialogue)
            if cases:
                cases_str = "\n".join(str(dict(r)) for r in cases)
                insight = self.analyzer.llm.generate(
                    "Compare this new case with historical patterns:\n"
                    f"New Case: {dialogue}\n\n"
                    f"Historical Similar Cases:\n{cases_str}\n\n"
                    "Identify any consistent patterns or anomalies.", temperature)
        return {"prediction": res["prediction"], "confidence": res["confidence"], "analysis": analysis,
                "historical_insight": insight}
