/*
 * Job types the CPU engine may hold: those of processes outside the device subset and of instances
 * handed off to the engine.  JOB_BATCH:ACTIVATE of such a type stays with the engine
 * (JobBatchActivateProcessor.java:60-143 activates across every instance in JOB_ACTIVATABLE order,
 * and the adapter does not read the engine's rows).  Not compiled in this image (no JDK).
 */
package io.camunda.zeebe.zbhip;

import io.camunda.zeebe.engine.state.instance.JobRecordValue;
import io.camunda.zeebe.protocol.ZbColumnFamilies;
import java.nio.charset.StandardCharsets;
import java.util.HashSet;
import java.util.Set;
import java.util.regex.Matcher;
import java.util.regex.Pattern;
import org.agrona.concurrent.UnsafeBuffer;

final class JobTypes {
  static final int JOBS_COLUMN_FAMILY = ZbColumnFamilies.JOBS.ordinal();
  // zeebe:taskDefinition type="..." (static types; `=` expressions are refused by the compiler anyway)
  private static final Pattern TYPE = Pattern.compile("taskDefinition[^>]*?\\stype=\"([^\"=][^\"]*)\"");

  private JobTypes() {}

  static Set<String> of(final byte[] bpmnXml) {
    final Set<String> out = new HashSet<>();
    final Matcher m = TYPE.matcher(new String(bpmnXml, StandardCharsets.UTF_8));
    while (m.find()) {
      out.add(m.group(1));
    }
    return out;
  }

  // <message name="..."> (static names; the subset of the device's message catch events)
  private static final Pattern MESSAGE = Pattern.compile("<(?:\\w+:)?message\\b[^>]*?\\sname=\"([^\"=][^\"]*)\"");

  /** Static message names a BPMN XML declares (config 5: the PUBLISH commands the device takes). */
  static Set<String> messageNames(final byte[] bpmnXml) {
    final Set<String> out = new HashSet<>();
    final Matcher m = MESSAGE.matcher(new String(bpmnXml, StandardCharsets.UTF_8));
    while (m.find()) {
      out.add(m.group(1));
    }
    return out;
  }

  // <startEvent ...><messageEventDefinition ... messageRef="..."> and <message id="..." name="...">
  private static final Pattern START_REF = Pattern.compile(
      "<(?:\\w+:)?startEvent\\b[^>]*>\\s*<(?:\\w+:)?messageEventDefinition\\b[^>]*?\\smessageRef=\"([^\"]*)\"");
  private static final Pattern MESSAGE_ID_NAME =
      Pattern.compile("<(?:\\w+:)?message\\b([^>]*)>");
  private static final Pattern ATTR_ID = Pattern.compile("\\sid=\"([^\"]*)\"");
  private static final Pattern ATTR_NAME = Pattern.compile("\\sname=\"([^\"]*)\"");

  /**
   * Message names of the message start events a BPMN XML declares: a publish of such a name starts
   * instances (MessagePublishProcessor.correlateToMessageStartEvents, :157-180), so it is the engine's.
   */
  static Set<String> messageStartNames(final byte[] bpmnXml) {
    final String xml = new String(bpmnXml, StandardCharsets.UTF_8);
    final Set<String> refs = new HashSet<>();
    final Matcher r = START_REF.matcher(xml);
    while (r.find()) {
      refs.add(r.group(1));
    }
    final Set<String> out = new HashSet<>();
    final Matcher m = MESSAGE_ID_NAME.matcher(xml);
    while (m.find()) {
      final Matcher id = ATTR_ID.matcher(m.group(1));
      final Matcher name = ATTR_NAME.matcher(m.group(1));
      if (id.find() && name.find() && refs.contains(id.group(1))) {
        out.add(name.group(1));
      }
    }
    return out;
  }

  /** The job type of a JOBS column-family value (JobRecordValue, DbJobState.java:112-157). */
  static String typeOfJobsValue(final byte[] value) {
    final JobRecordValue v = new JobRecordValue();
    v.wrap(new UnsafeBuffer(value), 0, value.length);
    return v.getRecord().getType();
  }
}
