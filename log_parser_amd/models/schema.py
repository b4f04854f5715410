"""Data model: request, pattern library and analysis result.

The reference keeps these POJOs in an external artifact (``com.redhat.podmortem:common``,
``pom.xml:55-59``) whose source is unavailable; the schema here is inferred from call sites
(SURVEY.md §2.4):

* ``PodFailureData`` — ``Parse.java:4,45-57``, ``AnalysisService.java:53``
* ``PatternSet`` / ``Pattern`` / ``SecondaryPattern`` / ``SequencePattern`` / ``SequenceEvent`` /
  ``ContextExtraction`` — ``AnalysisService.java:55-113,132-156``, ``ScoringService.java:63-347``
* ``AnalysisResult`` / ``AnalysisMetadata`` / ``AnalysisSummary`` / ``MatchedEvent`` /
  ``EventContext`` — ``AnalysisService.java:100-121,166-215``

Compatibility decision: input accepts snake_case and camelCase keys; pattern
fields are emitted snake_case (the YAML spelling, ``docs/SCORING_ALGORITHM.md:29-33``),
analysis-result fields camelCase (Jackson bean default). Unknown fields are preserved on
patterns so that e.g. ``remediation`` round-trips into ``matchedPattern``.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from pydantic import AliasChoices, BaseModel, ConfigDict, Field


def _alias(snake: str, camel: str):
    return Field(default=None, validation_alias=AliasChoices(snake, camel), serialization_alias=snake)


class _PatternBase(BaseModel):
    model_config = ConfigDict(extra="allow", populate_by_name=True)


class PrimaryPattern(_PatternBase):
    regex: Optional[str] = None
    confidence: float = 0.0


class SecondaryPattern(_PatternBase):
    regex: Optional[str] = None
    weight: float = 0.0
    proximity_window: int = Field(default=0, validation_alias=AliasChoices("proximity_window", "proximityWindow"))


class SequenceEvent(_PatternBase):
    regex: Optional[str] = None


class SequencePattern(_PatternBase):
    description: Optional[str] = None
    bonus_multiplier: float = Field(default=0.0, validation_alias=AliasChoices("bonus_multiplier", "bonusMultiplier"))
    events: Optional[List[SequenceEvent]] = None


class ContextExtraction(_PatternBase):
    lines_before: int = Field(default=0, validation_alias=AliasChoices("lines_before", "linesBefore"))
    lines_after: int = Field(default=0, validation_alias=AliasChoices("lines_after", "linesAfter"))
    include_stack_trace: bool = Field(default=False, validation_alias=AliasChoices("include_stack_trace", "includeStackTrace"))


class Pattern(_PatternBase):
    id: Optional[str] = None
    name: Optional[str] = None
    severity: Optional[str] = None
    primary_pattern: Optional[PrimaryPattern] = Field(default=None, validation_alias=AliasChoices("primary_pattern", "primaryPattern"))
    secondary_patterns: Optional[List[SecondaryPattern]] = Field(default=None, validation_alias=AliasChoices("secondary_patterns", "secondaryPatterns"))
    sequence_patterns: Optional[List[SequencePattern]] = Field(default=None, validation_alias=AliasChoices("sequence_patterns", "sequencePatterns"))
    context_extraction: Optional[ContextExtraction] = Field(default=None, validation_alias=AliasChoices("context_extraction", "contextExtraction"))


class PatternSetMetadata(_PatternBase):
    library_id: Optional[str] = Field(default=None, validation_alias=AliasChoices("library_id", "libraryId"))


class PatternSet(_PatternBase):
    metadata: Optional[PatternSetMetadata] = None
    patterns: Optional[List[Pattern]] = None


# ---------------------------------------------------------------------------------------
# request
class ObjectMeta(BaseModel):
    model_config = ConfigDict(extra="allow")
    name: Optional[str] = None
    namespace: Optional[str] = None


class Pod(BaseModel):
    model_config = ConfigDict(extra="allow")
    metadata: Optional[ObjectMeta] = None


class PodFailureData(BaseModel):
    """``PodFailureData`` (pod + raw logs; events/spec are carried but unused, Parse.java:33-38)."""
    model_config = ConfigDict(extra="allow")
    pod: Optional[Pod] = None
    logs: Optional[str] = None


# ---------------------------------------------------------------------------------------
# result (camelCase, Jackson bean default)
class EventContext(BaseModel):
    matchedLine: Optional[str] = None
    linesBefore: Optional[List[str]] = None
    linesAfter: Optional[List[str]] = None


class MatchedEvent(BaseModel):
    lineNumber: int
    matchedPattern: Dict[str, Any]
    context: EventContext
    score: float


class AnalysisMetadata(BaseModel):
    processingTimeMs: int
    totalLines: int
    analyzedAt: str
    patternsUsed: List[Optional[str]]


class AnalysisSummary(BaseModel):
    significantEvents: int
    highestSeverity: Optional[str]
    severityDistribution: Dict[str, int]


class AnalysisResult(BaseModel):
    analysisId: str
    metadata: AnalysisMetadata
    events: List[MatchedEvent]
    summary: AnalysisSummary


def pattern_to_json(p: Pattern) -> Dict[str, Any]:
    """Echo of the full pattern object (snake_case, nulls kept like Jackson's default)."""
    return p.model_dump(by_alias=True, exclude_none=False)
