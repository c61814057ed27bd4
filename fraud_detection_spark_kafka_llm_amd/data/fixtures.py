"""Golden fixtures derived from the reference.

``SCAM_SAMPLE`` is the usage-example dialogue at /root/reference/utils/agent_api.py:224; the expected
values are those of the shipped ``dialogue_classification_model`` (HashingTF 10000 -> IDF -> LR).
"""

SCAM_SAMPLE = (
    'Innocent: Hello.  Suspect: Hello, this is Officer Rachel Johnson from the Social Security '
    "Administration. We've been trying to reach you about a serious issue with your social security "
    "number. It's been flagged for suspicious activity and we need to verify some information to avoid "
    "any further complications. Can you please confirm your social security number for me? Innocent: I'm "
    "not giving out my social security number over the phone. How do I know you're really from the Social"
    ' Security Administration? Can you provide me with a call-back number and a reference number for this'
    " case so I can verify it? Suspect: I understand your concern, ma'am. However, I need to inform you "
    "that this is an urgent matter and we can't afford to delay. Your social security number is at risk "
    "of being suspended due to fraudulent activity. If we don't verify the information immediately, it "
    "will be deactivated and you'll face severe consequences, including legal action. I'm not authorized "
    'to provide a call-back number, but I can give you a reference number: SSA-123456789. You can verify '
    "it on the SSA website. But please, ma'am, time is of the essence. Can you just confirm your social "
    "security number so we can resolve this issue? Innocent: I'm not buying it. If this is a legitimate "
    "issue, I should be able to verify it through the SSA's official website or by visiting a local "
    "office. I'm not giving out my social security number to someone who calls me out of the blue, "
    "regardless of the reference number. I think this is a scam. Suspect: Ma'am, I understand your "
    "skepticism, but I assure you, this is a legitimate issue. You're not taking this seriously, and "
    "that's putting your social security benefits at risk. If you don't cooperate, you'll be the one "
    "who's responsible for the consequences. You're going to regret not taking action when you had the "
    "chance. Let me transfer you to my supervisor, he'll explain the situation to you. Maybe you'll "
    "listen to him. Hold for just a moment, please. Innocent: No, I don't think so. I'm not going to hold"
    " for anyone. I'm going to hang up and report this to the real Social Security Administration. This "
    'sounds like a scam to me. Goodbye.'
)

BENIGN_SAMPLE = ("Innocent: Hello. Suspect: Hi, this is Dr. Smith's office calling to confirm your appointment "
                 "scheduled for Tuesday at 3 pm. Innocent: Thanks, see you then.")

# (text, margin, P(scam), prediction) for the shipped model
GOLDEN = [
    ("scam", 23.20628005344286, 0.9999999999165088, 1.0),
    ("benign", -10.094201159284516, 4.13167538969518e-05, 0.0),
    ("empty", -7.218662911169931, 0.000732244982553525, 0.0),
]

# murmur3 (seed 42) HashingTF buckets at numFeatures=10000
BUCKETS_10000 = {"innocent": 2833, "suspect": 9168, "hello": 9889, "": 3372, "verify": 336, "social": 823,
                 "scam": 874, "number": 8519, "im": 3623}


def golden_text(name: str) -> str:
    return {"scam": SCAM_SAMPLE, "benign": BENIGN_SAMPLE, "empty": ""}[name]
